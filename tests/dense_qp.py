"""Independent dense solve of the DCM-MPC QP (test infrastructure).

Given the active set, the QP optimum solves one equality-constrained KKT system; we build it
densely over z = (xi_1..xi_N, r_0..r_{N-1}) and solve it with scipy/numpy LU plus iterative
refinement in extended precision (residuals in np.longdouble), so its error is far below the
1e-9 parity bar.  The active set is taken from a candidate solution and then *verified*: the
dense solution must be primal feasible and its multipliers nonnegative, otherwise the check
fails — so this is a full optimality certificate, independent of the IPM.
"""
import numpy as np


def kkt_solve(prob, i, active, q=(1e2, 1e2), rw=(1.0, 1.0), pw=(1e3, 1e3), dt=0.02):
    A, bb, m = prob["A"][i], prob["b"][i], prob["nfacets"][i]
    om, xi0 = prob["omega"][i], prob["xi_init"][i]
    xr, rr = prob["xi_ref"][i], prob["vrp_ref"][i]
    N = om.shape[0]
    be = dt * om
    al = 1.0 + be
    nx, nz = 2 * N, 4 * N
    H = np.zeros((nz, nz))
    g = np.zeros(nz)
    for j in range(1, N + 1):
        w = pw if j == N else q
        for c in range(2):
            H[2 * (j - 1) + c, 2 * (j - 1) + c] = w[c]
            g[2 * (j - 1) + c] = -w[c] * xr[j, c]
    for k in range(N):
        for c in range(2):
            H[nx + 2 * k + c, nx + 2 * k + c] = rw[c]
            g[nx + 2 * k + c] = -rw[c] * rr[k, c]
    C, d = [], []
    for k in range(N):          # xi_{k+1} - al_k xi_k + be_k r_k = 0 (al_0 xi_0 moved to rhs)
        for c in range(2):
            row = np.zeros(nz)
            row[2 * k + c] = 1.0
            if k > 0:
                row[2 * (k - 1) + c] -= al[k]
            row[nx + 2 * k + c] += be[k]
            C.append(row)
            d.append(al[k] * xi0[c] if k == 0 else 0.0)
    act_idx = []
    for k in range(N):
        for f in range(m[k]):
            if active[k, f]:
                row = np.zeros(nz)
                row[nx + 2 * k:nx + 2 * k + 2] = A[k, f]
                C.append(row)
                d.append(bb[k, f])
                act_idx.append((k, f))
    C = np.array(C)
    d = np.array(d)
    nc = C.shape[0]
    K = np.block([[H, C.T], [C, np.zeros((nc, nc))]])
    rhs = np.concatenate([-g, d])
    Kl, rl = K.astype(np.longdouble), rhs.astype(np.longdouble)
    x = np.linalg.solve(K, rhs).astype(np.longdouble)
    for _ in range(5):
        res = rl - Kl @ x
        x = x + np.linalg.solve(K, res.astype(np.float64)).astype(np.longdouble)
    x = x.astype(np.float64)
    z = x[:nz]
    xi = np.vstack([xi0[None, :], z[:nx].reshape(N, 2)])
    r = z[nx:].reshape(N, 2)
    lam = x[nz + 2 * N:]          # multipliers of the active rows (KKT sign: H z + C^T y = -g)
    return xi, r, lam, act_idx


def certify(prob, i, xi_c, r_c, thresholds=(1e-9, 1e-8, 1e-7, 1e-6, 1e-5)):
    """Dense optimality certificate around a candidate (xi_c, r_c): returns (xi, r) of the exact
    optimum.  The active set is guessed from the candidate's slacks with increasing thresholds;
    a guess is accepted only if the dense solution is primal feasible and every multiplier is
    nonnegative (then it IS the unique optimum of the strictly convex QP)."""
    A, bb, m = prob["A"][i], prob["b"][i], prob["nfacets"][i]
    mask = np.arange(A.shape[1])[None, :] < m[:, None]
    viol = np.einsum("kfj,kj->kf", A, r_c) - bb
    for thr in thresholds:
        active = (viol > -thr) & mask
        xi, r, lam, _ = kkt_solve(prob, i, active)
        v2 = (np.einsum("kfj,kj->kf", A, r) - bb)[mask]
        feasible = v2.size == 0 or v2.max() <= 1e-12
        # with the sign convention of kkt_solve the inequality multipliers are y >= 0
        if feasible and (lam.size == 0 or lam.min() >= -1e-10):
            return xi, r
    raise AssertionError(f"no certified active set for problem {i}")
