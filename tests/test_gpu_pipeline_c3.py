"""configs[2] at its full size (BASELINE.json: batch 65 536 DCM-MPC QPs + QuinticSpline swing feet
+ ConvexHullHelper constraints on one MI355X): the bench's c3 step (bench.py --workload c3) end to
end on the device, under size-independent properties, plus a 256-problem subset bit for bit
against the oracle's C batch drivers.

Step: ConvexHullHelper on every phase polygon (blf_hull2d_hrep, 589 824 polygons), the QPs read
their knots' constraints from that phase table (blf_dcm_mpc_solve_phased), the swing splines
(blf_quintic_fit + blf_quintic_eval, 32 queries each).

Properties (every problem):
  * status 0 (solved) and polished (certified optimum);
  * primal feasibility of the returned VRPs against the window's support polygons, A r <= b + 1e-12
    (the polygons of ContactPhaseList.cpp:16-84 at the knots' times, ContactList.cpp:190-202);
  * the DCM trajectory is the reference Euler step of its VRPs, xi_{k+1} = xi_k + (w xi_k - w r_k) dt
    (ForwardEuler.tpp:37-45 over LinearTimeInvariantSystem.cpp:71), to 1e-12;
  * the splines interpolate their knots: position, velocity, acceleration at every knot time.
"""
import numpy as np
import pytest
import torch

from blf import native
from blf import problems as P

pytestmark = pytest.mark.gpu
B, N, Q = 65536, 100, 32


@pytest.fixture(scope="module")
def c3(handle):
    prob = P.make_batch(B, horizon=N, n_footsteps=6, seed=P.SEED)
    dev = lambda k: torch.from_numpy(np.ascontiguousarray(prob[k])).cuda()
    table = handle.phase_table(dev("nphases"), dev("phase_begin"), dev("phase_end"),
                               dev("phase_corners"), dev("phase_ncorners"), ref=dev("phase_ref"))
    params = native.default_params(N)
    qp = handle.dcm_mpc_solve_phased(table, 0, dev("xi_init"), dev("omega"), params)
    kt, kp, tq = (torch.from_numpy(a).cuda() for a in P.swing_splines(prob, queries=Q))
    coeffs = handle.quintic_fit(kt, kp)
    sp = handle.quintic_eval(kt, coeffs, tq)
    torch.cuda.synchronize()
    return dict(prob=prob, table=table, qp=qp, kt=kt, kp=kp, tq=tq, coeffs=coeffs, sp=sp)


def test_c3_solved_and_certified(c3):
    qp = c3["qp"]
    assert int((qp["status"] != 0).sum()) == 0
    assert bool((qp["polished"] == 1).all())


def test_c3_primal_feasibility(handle, c3):
    w = handle.dcm_phase_expand(c3["table"], 0, c3["prob"]["dt"], N)
    r = c3["qp"]["vrp"]                                          # [B, N, 2]
    viol = (w["A"] * r[:, :, None, :]).sum(-1) - w["b"]          # [B, N, M]
    m = torch.arange(w["b"].shape[2], device=r.device)[None, None, :] < w["nfacets"][:, :, None]
    worst = float(torch.where(m, viol, torch.full_like(viol, -1.0)).max())
    assert worst <= 1e-12, worst


def test_c3_dcm_is_the_euler_rollout_of_the_vrps(c3):
    xi, r = c3["qp"]["xi"], c3["qp"]["vrp"]
    w = torch.from_numpy(c3["prob"]["omega"]).cuda()[:, :, None]
    dt = c3["prob"]["dt"]
    xk = xi[:, :-1]
    step = xk + (w * xk + (-w) * r) * dt                          # the reference's operation order
    err = float((step - xi[:, 1:]).abs().max())
    assert err <= 1e-12, err
    assert torch.equal(xi[:, 0], torch.from_numpy(c3["prob"]["xi_init"]).cuda())


def test_c3_splines_interpolate_their_knots(handle, c3):
    kt, kp, coeffs = c3["kt"], c3["kp"], c3["coeffs"]
    pva, idx = handle.quintic_eval(kt, coeffs, kt.contiguous())   # at the knot times
    torch.cuda.synchronize()
    # pva [S, K+1, 3, D] against the knots' (p, v, a) [S, K+1, 3, D]
    err = (pva - kp).abs()
    scale = kp.abs().clamp(min=1.0)
    assert float((err[:, :, 0] / scale[:, :, 0]).max()) <= 1e-12
    assert float((err[:, :, 1] / scale[:, :, 1]).max()) <= 1e-11
    assert float((err[:, :, 2] / scale[:, :, 2]).max()) <= 1e-9
    # knot indices at the knot times: the getPresentContact rule (the last knot with t_j <= t),
    # i.e. the knot itself (the evaluated segment is that index clamped to [0, K - 1])
    expect = torch.arange(kt.shape[1], dtype=torch.int32, device=idx.device)
    assert torch.equal(idx, expect[None, :].expand_as(idx))


def test_c3_subset_bitwise_vs_oracle(c3, oracle):
    prob, qp, sp = c3["prob"], c3["qp"], c3["sp"]
    idx = np.sort(np.random.default_rng(3).choice(B, 256, replace=False))
    Pn, C = prob["phase_corners"].shape[1:3]
    A, b, nf = oracle.hull2d_hrep_batch(prob["phase_corners"][idx].reshape(256 * Pn, C, 2),
                                        prob["phase_ncorners"][idx].reshape(256 * Pn), 8, threads=8)
    # the device table's polygons, bit for bit
    tab = c3["table"]
    it = torch.from_numpy(idx).cuda()
    np.testing.assert_array_equal(tab["phase_A"][it].cpu().numpy(), A.reshape(256, Pn, 8, 2))
    np.testing.assert_array_equal(tab["phase_b"][it].cpu().numpy(), b.reshape(256, Pn, 8))
    np.testing.assert_array_equal(tab["phase_nf"][it].cpu().numpy(), nf.reshape(256, Pn))
    otab = dict(nphases=prob["nphases"][idx], phase_begin=prob["phase_begin"][idx],
                phase_end=prob["phase_end"][idx], phase_A=A.reshape(256, Pn, 8, 2),
                phase_b=b.reshape(256, Pn, 8), phase_nf=nf.reshape(256, Pn),
                phase_ref=prob["phase_ref"][idx])
    w = oracle.dcm_phase_expand_batch(otab, 0, prob["dt"], N, threads=8)
    w.update(xi_init=np.ascontiguousarray(prob["xi_init"][idx]),
             omega=np.ascontiguousarray(prob["omega"][idx]))
    st, xi, vrp, iters = oracle.dcm_mpc_solve_batch(w, threads=8, device_batch=B)   # B-QP launch
    np.testing.assert_array_equal(qp["status"][it].cpu().numpy(), st)
    np.testing.assert_array_equal(qp["iters"][it].cpu().numpy(), iters)
    np.testing.assert_array_equal(qp["xi"][it].cpu().numpy(), xi)
    np.testing.assert_array_equal(qp["vrp"][it].cpu().numpy(), vrp)
    # the splines of the same problems (every swing of problem i is row s * B + i)
    kt, kp, tq = (a.cpu().numpy() for a in (c3["kt"], c3["kp"], c3["tq"]))
    S = kt.shape[0] // B
    rows = (np.arange(S)[:, None] * B + idx[None, :]).reshape(-1)
    coeffs, pva, kidx = oracle.quintic_batch(kt[rows], kp[rows], tq[rows], threads=8)
    np.testing.assert_array_equal(c3["coeffs"].cpu().numpy()[rows], coeffs)
    np.testing.assert_array_equal(sp[0].cpu().numpy()[rows], pva)
    np.testing.assert_array_equal(sp[1].cpu().numpy()[rows], kidx)
