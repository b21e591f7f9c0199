"""Independent reference solve of the DCM-MPC QP by a dual active-set method (test infrastructure).

tests/dense_qp.py certifies a candidate: it needs a candidate whose slacks identify the optimal
active set.  This module finds the optimum with no candidate at all, for the QPs the solver under
test may fail on (tests/golden/c5_hard_windows.npz): the QP is condensed onto the VRPs
r = (r_0..r_{N-1}) (xi = Phi xi_0 + Gamma r), and the strictly convex problem

    min 1/2 r^T H r + g^T r   s.t.   a_{k,i} . r_k <= b_{k,i}

is solved by the Goldfarb-Idnani dual method (Math. Programming 27 (1983) 1-33): start at the
unconstrained minimum, add the most violated facet, drop facets whose multiplier would turn
negative, until every facet holds.  Each step recomputes the QR factors of J^T N_A (J = L^{-T},
H = L L^T) from scratch: O(n |A|^2) per step, fine for N = 100.  The active set it ends with is then
handed to dense_qp.kkt_solve (extended-precision refinement) and certified there, so the returned
optimum does not depend on the rounding of the condensed form.
"""
import numpy as np

import dense_qp


def condensed(prob, i, q=(1e2, 1e2), rw=(1.0, 1.0), pw=(1e3, 1e3), dt=0.02):
    """H, g of the QP in r, and the affine map xi = x0 + G r (xi_1..xi_N stacked [N][2])."""
    om, xi0 = prob["omega"][i], prob["xi_init"][i]
    xr, rr = prob["xi_ref"][i], prob["vrp_ref"][i]
    N = om.shape[0]
    be = dt * om
    al = 1.0 + be
    n = 2 * N
    G = np.zeros((n, n))        # d xi_{k+1} / d r_j
    x0 = np.zeros(n)
    prev_x, prevG = xi0.copy(), np.zeros((2, n))
    for k in range(N):
        xk = al[k] * prev_x
        Gk = al[k] * prevG
        Gk[0, 2 * k] -= be[k]
        Gk[1, 2 * k + 1] -= be[k]
        x0[2 * k:2 * k + 2] = xk
        G[2 * k:2 * k + 2] = Gk
        prev_x, prevG = xk, Gk
    qd = np.array([q if k < N - 1 else pw for k in range(N)], dtype=float).reshape(n)
    H = G.T @ (qd[:, None] * G) + np.diag(np.tile(rw, N))
    g = G.T @ (qd * (x0 - xr[1:].reshape(n))) - np.tile(rw, N) * rr.reshape(n)
    return H, g, x0, G


def goldfarb_idnani(H, g, Nc, bc, max_steps=20000, tol=1e-12):
    """min 1/2 x^T H x + g^T x s.t. Nc^T x <= bc (columns of Nc are the constraint normals).
    Returns x, the active index list and the multipliers u >= 0 of the active constraints."""
    L = np.linalg.cholesky(H)
    J = np.linalg.inv(L).T                 # H^{-1} = J J^T
    x = -np.linalg.solve(H, g)
    act, u = [], np.zeros(0)
    scale = np.maximum(1.0, np.abs(bc))
    for _ in range(max_steps):
        s = (Nc.T @ x - bc) / scale
        s[act] = -np.inf
        p = int(np.argmax(s))
        if s[p] <= tol:
            return x, act, u
        npv = Nc[:, p]
        up = 0.0
        while True:
            d = J.T @ npv
            if act:
                Q, R = np.linalg.qr(J.T @ Nc[:, act], mode="complete")
                k = len(act)
                z = J @ (Q[:, k:] @ (Q[:, k:].T @ d))
                r = np.linalg.solve(R[:k, :k], Q[:, :k].T @ d)
            else:
                z, r = J @ (J.T @ npv), np.zeros(0)
            # the step enters with the violated constraint's multiplier growing: for A x <= b
            # the primal moves along -z
            t1, l = np.inf, -1
            for j in range(len(act)):
                if r[j] > 0 and u[j] / r[j] < t1:
                    t1, l = u[j] / r[j], j
            viol = npv @ x - bc[p]
            zz = z @ npv
            t2 = viol / zz if zz > 1e-300 else np.inf
            t = min(t1, t2)
            if t == np.inf:
                raise ValueError("infeasible QP")
            if t2 == np.inf:        # partial step in the dual only
                u = u - t * r
                up += t
                del act[l]
                u = np.delete(u, l)
                continue
            x = x - t * z
            u = u - t * r
            up += t
            if t2 <= t1:
                act.append(p)
                u = np.append(u, up)
                break
            del act[l]
            u = np.delete(u, l)
    raise RuntimeError("no convergence")


def solve(prob, i, **w):
    """The optimum (xi [N+1][2], r [N][2]) of problem i and its active set [N][M] (bool),
    certified by the dense extended-precision KKT solve of dense_qp."""
    A, bb, m = prob["A"][i], prob["b"][i], prob["nfacets"][i]
    N, M = bb.shape
    H, g, x0, G = condensed(prob, i, **w)
    cols, rhs, idx = [], [], []
    for k in range(N):
        for f in range(m[k]):
            c = np.zeros(2 * N)
            c[2 * k:2 * k + 2] = A[k, f]
            cols.append(c)
            rhs.append(bb[k, f])
            idx.append((k, f))
    Nc, bc = np.array(cols).T, np.array(rhs)
    r, act, u = goldfarb_idnani(H, g, Nc, bc)
    active = np.zeros((N, M), bool)
    for j in act:
        active[idx[j]] = True
    xi, rr, lam, _ = dense_qp.kkt_solve(prob, i, active, **w)
    mask = np.arange(M)[None, :] < m[:, None]
    v = (np.einsum("kfj,kj->kf", A, rr) - bb)[mask]
    assert v.size == 0 or v.max() <= 1e-9, ("reference optimum infeasible", v.max())
    assert lam.size == 0 or lam.min() >= -1e-6 * max(1.0, np.abs(lam).max()), ("negative multiplier", lam.min())
    return xi, rr, active, lam


def lq_solve_ld(prob, i, active, q=(1e2, 1e2), rw=(1.0, 1.0), pw=(1e3, 1e3), dt=0.02):
    """The optimum of problem i with the facets `active` [N][M] as equalities, by a Riccati
    recursion over the reduced inputs in extended precision (np.longdouble): at a knot with two
    active facets r_k is their vertex, with one r_k = p + t u on its line, with none r_k = u.  An
    algorithm independent of the solver under test and of dense_qp's LU, and exact to ~1e-18
    relative, so it resolves errors the dense solve's refinement cannot on the QPs whose
    multipliers reach 1e7.  Returns xi [N+1][2], r [N][2] (float64) and the multipliers [N][M]."""
    L = np.longdouble
    A, bb, m = prob["A"][i].astype(L), prob["b"][i].astype(L), prob["nfacets"][i]
    om = prob["omega"][i].astype(L)
    xr, rr = prob["xi_ref"][i].astype(L), prob["vrp_ref"][i].astype(L)
    N, M = bb.shape
    be = L(dt) * om
    al = 1 + be
    Q, R, PT = (np.diag(np.array(v, dtype=L)) for v in (q, rw, pw))
    base, Tm = [], []
    for k in range(N):
        idx = [f for f in range(m[k]) if active[k, f]]
        if len(idx) >= 2:
            a, e = A[k, idx[0]], A[k, idx[1]]
            det = a[0] * e[1] - a[1] * e[0]
            v = np.array([(bb[k, idx[0]] * e[1] - a[1] * bb[k, idx[1]]) / det,
                          (a[0] * bb[k, idx[1]] - bb[k, idx[0]] * e[0]) / det], dtype=L)
            base.append(v)
            Tm.append(np.zeros((2, 0), dtype=L))
        elif len(idx) == 1:
            a = A[k, idx[0]]
            aa = a @ a
            base.append(a * (bb[k, idx[0]] / aa))
            Tm.append(np.array([[-a[1]], [a[0]]], dtype=L) / np.sqrt(aa))
        else:
            base.append(np.zeros(2, dtype=L))
            Tm.append(np.eye(2, dtype=L))
    # backward: V_{k+1}(x) = 1/2 x^T S x + s^T x;  u_k = K_k x_k + f_k
    S, s = PT.copy(), -(PT @ xr[N])
    gains = [None] * N
    for k in range(N - 1, -1, -1):
        T, c = Tm[k], base[k]
        if T.shape[1]:
            Hu = T.T @ R @ T + be[k] ** 2 * (T.T @ S @ T)
            Hi = np.linalg.inv(Hu.astype(np.float64)).astype(L)
            for _ in range(3):   # Newton refinement of the small inverse in long double
                Hi = Hi + Hi @ (np.eye(Hu.shape[0], dtype=L) - Hu @ Hi)
            Kk = Hi @ (be[k] * al[k] * (T.T @ S))
            fk = -Hi @ (T.T @ R @ (c - rr[k]) - be[k] * (T.T @ (s - be[k] * (S @ c))))
        else:
            Kk, fk = np.zeros((0, 2), dtype=L), np.zeros(0, dtype=L)
        gains[k] = (Kk, fk)
        # closed loop: x' = F x + e, r = c + T (K x + f)
        F = al[k] * np.eye(2, dtype=L) - be[k] * (T @ Kk)
        e = -be[k] * (c + T @ fk)
        G, h = T @ Kk, c + T @ fk - rr[k]    # r - rref = G x + h
        Sn = F.T @ S @ F + G.T @ R @ G
        sn = F.T @ (S @ e + s) + G.T @ R @ h
        if k >= 1:
            Sn, sn = Sn + Q, sn - Q @ xr[k]
        S, s = Sn, sn
    xi = np.zeros((N + 1, 2), dtype=L)
    xi[0] = prob["xi_init"][i].astype(L)
    r = np.zeros((N, 2), dtype=L)
    for k in range(N):
        Kk, fk = gains[k]
        r[k] = base[k] + Tm[k] @ (Kk @ xi[k] + fk)
        xi[k + 1] = al[k] * xi[k] - be[k] * r[k]
    # costates nu_N = P (xi_N - ref), nu_k = Q (xi_k - ref) + alpha_k nu_{k+1}; multipliers from
    # beta_k nu_{k+1} - R (r_k - rref_k) = A_act^T lam
    nu = np.zeros((N + 1, 2), dtype=L)
    nu[N] = PT @ (xi[N] - xr[N])
    for k in range(N - 1, 0, -1):
        nu[k] = Q @ (xi[k] - xr[k]) + al[k] * nu[k + 1]
    lam = np.zeros((N, M))
    for k in range(N):
        g = be[k] * nu[k + 1] - R @ (r[k] - rr[k])
        idx = [f for f in range(m[k]) if active[k, f]]
        if len(idx) == 1:
            a = A[k, idx[0]]
            lam[k, idx[0]] = float((a @ g) / (a @ a))
        elif len(idx) >= 2:
            a, e = A[k, idx[0]], A[k, idx[1]]
            det = a[0] * e[1] - a[1] * e[0]
            lam[k, idx[0]] = float((g[0] * e[1] - e[0] * g[1]) / det)
            lam[k, idx[1]] = float((a[0] * g[1] - g[0] * a[1]) / det)
    return xi.astype(np.float64), r.astype(np.float64), lam
