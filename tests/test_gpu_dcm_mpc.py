"""GPU parity of the batched DCM-MPC QP (blf_dcm_mpc_solve) against the CPU oracle.

The oracle (oracle/blf_oracle.c:orc_dcm_mpc_solve) and the kernel evaluate the same IPM in the
same expression order with FMA contraction off on both sides, so the bar is bit equality of
xi, vrp, status and iteration count.  The north-star tolerance (fp64 trajectory error < 1e-9)
is asserted as well, as the floor every run must clear.
"""
import numpy as np
import pytest
import torch

from blf import problems as P
from blf import native

pytestmark = pytest.mark.gpu
TOL = 1e-9   # north_star: fp64 trajectory error < 1e-9 vs the reference CPU path


def _to_dev(prob, keys=("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets")):
    return {k: torch.from_numpy(np.ascontiguousarray(prob[k])).cuda() for k in keys}


def _gpu_problem(handle, prob):
    dev = _to_dev(prob, ("xi_init", "omega", "xi_ref", "vrp_ref"))
    corners = torch.from_numpy(prob["corners"]).cuda()
    ncorners = torch.from_numpy(prob["ncorners"]).cuda()
    A, b, nf = handle.assemble_constraints(corners, ncorners)
    dev.update(A=A, b=b, nfacets=nf)
    return dev


@pytest.mark.parametrize("horizon,footsteps,batch", [(100, 6, 96), (50, 4, 64), (130, 8, 32)])
def test_dcm_mpc_matches_oracle_bitwise(handle, oracle, horizon, footsteps, batch):
    prob = P.make_batch(batch, horizon=horizon, n_footsteps=footsteps, seed=11)
    dev = _gpu_problem(handle, prob)
    # the device hull feeds the QP; the oracle gets the same A, b, nfacets
    host = dict(prob)
    for k in ("A", "b", "nfacets"):
        host[k] = dev[k].cpu().numpy()
    out = handle.dcm_mpc_solve(dev)
    torch.cuda.synchronize()
    pol_o = np.zeros(batch, np.int32)
    st_o, xi_o, vrp_o, it_o, _ = oracle.dcm_mpc_solve_batch_warm(host, threads=8, polished=pol_o)
    xi_g, vrp_g = out["xi"].cpu().numpy(), out["vrp"].cpu().numpy()
    st_g, it_g = out["status"].cpu().numpy(), out["iters"].cpu().numpy()
    assert (st_g == 0).all(), st_g
    assert (st_o == 0).all()
    np.testing.assert_array_equal(it_g, it_o)
    np.testing.assert_array_equal(out["polished"].cpu().numpy(), pol_o)
    assert pol_o.all()   # every default solve ends in the certified active-set polish
    assert np.abs(xi_g - xi_o).max() <= TOL
    assert np.abs(vrp_g - vrp_o).max() <= TOL
    np.testing.assert_array_equal(xi_g, xi_o)
    np.testing.assert_array_equal(vrp_g, vrp_o)


def test_dcm_mpc_solution_properties(handle):
    """Size-independent checks on a larger batch: feasibility, the reference Euler step between
    consecutive knots, and xi_0 = xi_init."""
    B, N = 2048, 100
    prob = P.make_batch(B, horizon=N, n_footsteps=6, seed=5)
    dev = _gpu_problem(handle, prob)
    out = handle.dcm_mpc_solve(dev)
    xi, vrp = out["xi"], out["vrp"]
    assert (out["status"] == 0).all()
    assert torch.equal(xi[:, 0], dev["xi_init"])
    A, b, nf = dev["A"], dev["b"], dev["nfacets"]
    viol = torch.einsum("bkij,bkj->bki", A, vrp) - b
    mask = torch.arange(A.shape[2], device=A.device)[None, None, :] < nf[:, :, None]
    assert viol[mask].max().item() <= 1e-12
    w = dev["omega"]
    step = xi[:, :-1] + (w[..., None] * xi[:, :-1] + (-w[..., None]) * vrp) * 0.02
    assert (step - xi[:, 1:]).abs().max().item() <= 1e-12


def test_dcm_mpc_edge_cases(handle, oracle):
    B, N = 8, 20
    prob = P.make_batch(B, horizon=N, n_footsteps=4, seed=3)
    host = oracle.assemble_constraints(prob)
    # problem 1: no constraints at all (equality-only QP); problem 2: a bad facet count
    host["nfacets"][1, :] = 0
    host["nfacets"][2, 5] = 9
    dev = _to_dev(host)
    out = handle.dcm_mpc_solve(dev)
    st_o, xi_o, vrp_o, it_o = oracle.dcm_mpc_solve_batch(host, threads=1)
    st_g = out["status"].cpu().numpy()
    np.testing.assert_array_equal(st_g, st_o)
    assert st_g[2] == native.QP_BAD_FACETS and st_g[1] == native.QP_SOLVED
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), it_o)
    np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi_o)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp_o)


def test_dcm_mpc_horizon_one_and_empty_batch(handle, oracle):
    prob = P.make_batch(4, horizon=1, n_footsteps=2, seed=1)
    host = oracle.assemble_constraints(prob)
    out = handle.dcm_mpc_solve(_to_dev(host))
    st_o, xi_o, vrp_o, it_o = oracle.dcm_mpc_solve_batch(host, threads=1)
    np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi_o)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp_o)
    empty = {k: v[:0] for k, v in _to_dev(host).items()}
    res = handle.dcm_mpc_solve(empty)
    assert res["xi"].shape[0] == 0


def test_dcm_mpc_rejects_bad_params(handle):
    prob = P.make_batch(2, horizon=10, n_footsteps=4, seed=1)
    dev = _gpu_problem(handle, prob)
    p = native.default_params(10, max_facets=8, dt=-1.0)
    with pytest.raises(native.BlfError):
        handle.dcm_mpc_solve(dev, params=p)


def _bitwise_vs_oracle(handle, oracle, host, params=None, oparams=None):
    out = handle.dcm_mpc_solve(_to_dev(host), params=params)
    st_o, xi_o, vrp_o, it_o = oracle.dcm_mpc_solve_batch(host, params=oparams, threads=8)
    np.testing.assert_array_equal(out["status"].cpu().numpy(), st_o)
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), it_o)
    np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi_o)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp_o)
    return st_o, it_o


@pytest.mark.parametrize("horizon", [63, 64, 65, 126, 127, 128, 129, 200, 256, 300])
def test_dcm_mpc_wavefront_boundaries(handle, oracle, horizon):
    """Horizons around the 64-knot wavefront boundaries and multi-wavefront workgroups (the
    scans' cross-wavefront steps, padding wavefronts of the 256 / 512-thread variants)."""
    prob = P.make_batch(12, horizon=horizon, n_footsteps=8, seed=horizon)
    host = oracle.assemble_constraints(prob)
    st, _ = _bitwise_vs_oracle(handle, oracle, host)
    assert (st == 0).all()


def _bounding_boxes(prob):
    """Every knot's support polygon replaced by its axis-aligned bounding box: 4 facets, so the
    M = 4 kernel instantiation gets a plan it can hold (staggered double support needs 6)."""
    c, n = prob["corners"], prob["ncorners"]
    lo = np.where(np.arange(c.shape[2])[None, None, :, None] < n[..., None, None], c, np.inf).min(2)
    hi = np.where(np.arange(c.shape[2])[None, None, :, None] < n[..., None, None], c, -np.inf).max(2)
    box = np.zeros_like(c)
    box[:, :, 0] = lo
    box[:, :, 1] = np.stack([hi[..., 0], lo[..., 1]], -1)
    box[:, :, 2] = hi
    box[:, :, 3] = np.stack([lo[..., 0], hi[..., 1]], -1)
    return dict(prob, corners=box, ncorners=np.full_like(n, 4))


@pytest.mark.parametrize("M", [4, 6])
def test_dcm_mpc_fewer_facet_slots(handle, oracle, M):
    prob = P.make_batch(16, horizon=80, n_footsteps=6, seed=M)
    if M == 4:
        prob = _bounding_boxes(prob)
    host = oracle.assemble_constraints(prob, max_facets=M)
    assert (host["nfacets"] >= 3).all() and (host["nfacets"] <= M).all()
    p = native.default_params(80, max_facets=M)
    op = oracle.default_params(80, max_facets=M)
    _bitwise_vs_oracle(handle, oracle, host, p, op)


def test_dcm_mpc_other_weights_and_iteration_cap(handle, oracle):
    prob = P.make_batch(16, horizon=60, n_footsteps=5, seed=77)
    host = oracle.assemble_constraints(prob)
    kw = dict(w_xi=(10.0, 30.0), w_vrp=(2.0, 0.5), w_terminal=(100.0, 500.0), dt=0.015)
    _bitwise_vs_oracle(handle, oracle, host, native.default_params(60, **kw),
                       oracle.default_params(60, **kw))
    # a cap below the iterations needed: MAX_ITER with iters == cap on both sides (the interior
    # point method alone, and with the polish, whose first successes come after 2 iterations)
    st, it = _bitwise_vs_oracle(handle, oracle, host,
                                native.default_params(60, max_iter=4, tol_polish=0.0),
                                oracle.default_params(60, max_iter=4, tol_polish=0.0))
    assert (st == native.QP_MAX_ITER).all() and (it == 4).all()
    # with the polish on, the active-set start runs before the cap applies
    st, it = _bitwise_vs_oracle(handle, oracle, host, native.default_params(60, max_iter=1),
                                oracle.default_params(60, max_iter=1))
    assert np.isin(st, (0, native.QP_MAX_ITER)).all() and (it <= 1).all()


def test_dcm_mpc_infeasible_and_nonfinite_inputs(handle, oracle):
    prob = P.make_batch(6, horizon=40, n_footsteps=4, seed=13)
    host = oracle.assemble_constraints(prob)
    # problem 0, knot 10: two opposite half-planes that exclude each other (empty polygon)
    host["A"][0, 10, :2] = [[1.0, 0.0], [-1.0, 0.0]]
    host["b"][0, 10, :2] = [-1.0, -1.0]
    host["nfacets"][0, 10] = 2
    # problem 1: a NaN CoM frequency
    host["omega"][1, 3] = np.nan
    st, _ = _bitwise_vs_oracle(handle, oracle, host)
    assert st[0] != native.QP_SOLVED and st[1] != native.QP_SOLVED
    assert (st[2:] == native.QP_SOLVED).all()


def test_dcm_mpc_ipm_only_matches_oracle_bitwise(handle, oracle):
    """tol_polish = 0: the interior point method alone (stops at mu <= tol_mu), bit for bit."""
    B, N = 48, 100
    prob = P.make_batch(B, horizon=N, n_footsteps=6, seed=21)
    dev = _gpu_problem(handle, prob)
    host = dict(prob)
    for k in ("A", "b", "nfacets"):
        host[k] = dev[k].cpu().numpy()
    out = handle.dcm_mpc_solve(dev, params=native.default_params(N, tol_polish=0.0))
    pol_o = np.ones(B, np.int32)
    st_o, xi_o, vrp_o, it_o, _ = oracle.dcm_mpc_solve_batch_warm(
        host, params=oracle.default_params(N, tol_polish=0.0), threads=8, polished=pol_o)
    assert (st_o == 0).all() and not pol_o.any()
    assert not out["polished"].any()
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), it_o)
    np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi_o)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp_o)


def test_dcm_mpc_gpu_against_dense_certificate(handle):
    """The device solutions against the independent dense KKT optimum (tests/dense_qp.py): the
    polished optimum is exact to rounding, far inside north_star's 1e-9."""
    import dense_qp
    B, N = 512, 100
    prob = P.make_batch(B, horizon=N, n_footsteps=6, seed=33)
    dev = _gpu_problem(handle, prob)
    out = handle.dcm_mpc_solve(dev)
    host = dict(prob)
    for k in ("A", "b", "nfacets"):
        host[k] = dev[k].cpu().numpy()
    xi, vrp = out["xi"].cpu().numpy(), out["vrp"].cpu().numpy()
    assert (out["status"] == 0).all() and out["polished"].all()
    worst = 0.0
    for i in range(0, B, 8):
        xd, rd = dense_qp.certify(host, i, xi[i], vrp[i])
        worst = max(worst, np.abs(xd - xi[i]).max(), np.abs(rd - vrp[i]).max())
    assert worst < 1e-12, worst


def test_dcm_mpc_polish_refusal_matches_oracle_bitwise(handle, oracle):
    """Duplicated facet rows (parallel or more than two active facets): the polish's refusal path
    and the interior point method that then finishes alone, bit for bit with the oracle."""
    prob = oracle.assemble_constraints(P.make_batch(8, horizon=40, n_footsteps=4, seed=81))
    for q in range(8):
        for k in range(40):
            m = prob["nfacets"][q, k]
            c = min(2, 8 - m)
            prob["A"][q, k, m:m + c] = prob["A"][q, k, 0]
            prob["b"][q, k, m:m + c] = prob["b"][q, k, 0]
            prob["nfacets"][q, k] = m + c
    dev = _to_dev(prob)
    out = handle.dcm_mpc_solve(dev)
    pol_o = np.zeros(8, np.int32)
    st_o, xi_o, vrp_o, it_o, _ = oracle.dcm_mpc_solve_batch_warm(prob, threads=4, polished=pol_o)
    assert not pol_o.all()
    np.testing.assert_array_equal(out["status"].cpu().numpy(), st_o)
    np.testing.assert_array_equal(out["polished"].cpu().numpy(), pol_o)
    np.testing.assert_array_equal(out["iters"].cpu().numpy(), it_o)
    np.testing.assert_array_equal(out["xi"].cpu().numpy(), xi_o)
    np.testing.assert_array_equal(out["vrp"].cpu().numpy(), vrp_o)


@pytest.mark.parametrize("horizon", [40, 64])
def test_dcm_mpc_fused_stage2_equals_two_launches(handle, oracle, horizon):
    """Small batches with N <= 64 run the IPM's stage 2 inside the active-set kernel's workgroup
    (dcm_mpc_cold_fused_kernel, one launch); blf_set_qp_launch_mode(fuse_stage2 = 0) keeps the two
    launches.  Both
    give the oracle's bits, with QPs handed over (duplicated facet rows: the polish refuses) and
    an infeasible one."""
    B = 8
    prob = oracle.assemble_constraints(P.make_batch(B, horizon=horizon, n_footsteps=4, seed=82))
    for q in range(0, B, 2):
        for k in range(horizon):
            m = prob["nfacets"][q, k]
            c = min(2, 8 - m)
            prob["A"][q, k, m:m + c] = prob["A"][q, k, 0]
            prob["b"][q, k, m:m + c] = prob["b"][q, k, 0]
            prob["nfacets"][q, k] = m + c
    prob["A"][1, 10, :2] = [[1.0, 0.0], [-1.0, 0.0]]   # problem 1: an empty polygon at knot 10
    prob["b"][1, 10, :2] = [-1.0, -1.0]
    prob["nfacets"][1, 10] = 2
    dev = _to_dev(prob)
    res = {}
    try:
        for mode in ("1", "0"):
            native.set_qp_launch_mode(fuse_stage2=int(mode))
            out = handle.dcm_mpc_solve(dev, lambda_out=True)
            torch.cuda.synchronize()
            res[mode] = {k: v.cpu().numpy().copy() for k, v in out.items()}
    finally:
        native.set_qp_launch_mode(fuse_stage2=1)
    pol_o = np.zeros(B, np.int32)
    st_o, xi_o, vrp_o, it_o, lam_o = oracle.dcm_mpc_solve_batch_warm(prob, threads=4, polished=pol_o)
    assert not pol_o.all() and (st_o[0::2] == 0).all() and st_o[1] != 0
    for mode, r in res.items():
        for k, ref in (("status", st_o), ("polished", pol_o), ("iters", it_o), ("xi", xi_o),
                       ("vrp", vrp_o), ("lam", lam_o)):
            np.testing.assert_array_equal(r[k], ref, err_msg=f"{k} fuse={mode}")


@pytest.mark.parametrize("horizon,footsteps", [(100, 6), (50, 4), (128, 8), (126, 8), (65, 4)])
def test_dcm_mpc_active_set_kernel_and_single_kernel(handle, oracle, horizon, footsteps):
    """The default path for N <= 128 (csrc/dcm_mpc_as.hip: one wavefront per QP, knot pairs per
    lane, then the IPM kernel's stage 2 on the QPs it hands over) and the IPM kernel alone
    (blf_set_qp_launch_mode(single_kernel = 1), the wavefront scan tree) each equal the oracle evaluated the same way
    bit for bit, cold and warm; the two trees agree to rounding (both are certified optima)."""
    B = 1024
    prob = P.make_batch(B, horizon=horizon, n_footsteps=footsteps, seed=5)
    dev = _gpu_problem(handle, prob)
    host = dict(prob)
    for k in ("A", "b", "nfacets"):
        host[k] = dev[k].cpu().numpy()
    res = {}
    try:
        for mode in ("0", "1"):
            native.set_qp_launch_mode(single_kernel=int(mode))
            prm_o = oracle.default_params(horizon, single_kernel=int(mode))
            out = handle.dcm_mpc_solve(dev, lambda_out=True)
            torch.cuda.synchronize()
            cold = {k: v.cpu().numpy().copy() for k, v in out.items()}
            pol = np.zeros(B, np.int32)
            pas = np.zeros(B, np.int32)
            st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(host, params=prm_o, threads=8, polished=pol,
                                                                   passes=pas)
            for k, ref in (("status", st), ("xi", xi), ("vrp", vrp), ("iters", it), ("lam", lam),
                           ("polished", pol), ("passes", pas)):
                np.testing.assert_array_equal(cold[k], ref, err_msg=f"cold {k} mode {mode}")
            warm = dict(vrp=out["vrp"], lam=out["lam"], shift=1, floor=1e-3)
            outw = handle.dcm_mpc_solve(dev, warm=warm, lambda_out=True)
            torch.cuda.synchronize()
            pol = np.zeros(B, np.int32)
            pas = np.zeros(B, np.int32)
            st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(
                host, vrp_ws=cold["vrp"], lam_ws=cold["lam"], shift=1, floor=1e-3, params=prm_o,
                threads=8, polished=pol, passes=pas)
            for k, ref in (("status", st), ("xi", xi), ("vrp", vrp), ("iters", it), ("lam", lam),
                           ("polished", pol), ("passes", pas)):
                np.testing.assert_array_equal(outw[k].cpu().numpy(), ref, err_msg=f"warm {k} mode {mode}")
            if mode == "0":   # the active-set kernels: a cold start runs the fp32 search first
                assert (cold["passes"] >= 1).all() and (outw["passes"].cpu().numpy() >= 1).all()
            else:             # the interior point kernel alone
                assert (cold["passes"] == 0).all()
            res[mode] = cold
    finally:
        native.set_qp_launch_mode(single_kernel=0)
    assert (res["0"]["status"] == 0).all()
    assert np.abs(res["0"]["xi"] - res["1"]["xi"]).max() <= 1e-12
    assert np.abs(res["0"]["vrp"] - res["1"]["vrp"]).max() <= 1e-12


def test_bench_batch_bitwise(handle, oracle):
    """The bench's own configs[1] launch (bench.py: 4096 QPs, horizon 100, 6-footstep plans of seed
    P.SEED, support polygons assembled on the device): every one of the 4096 solves bit for bit
    against the oracle evaluated for that launch size, all certified, passes included."""
    B = 4096
    prob = P.make_batch(B, horizon=100, n_footsteps=6, seed=P.SEED)
    dev = _gpu_problem(handle, prob)
    host = dict(prob)
    for k in ("A", "b", "nfacets"):
        host[k] = dev[k].cpu().numpy()
    out = handle.dcm_mpc_solve(dev)
    torch.cuda.synchronize()
    pol, pas = np.zeros(B, np.int32), np.zeros(B, np.int32)
    st, xi, vrp, it, _ = oracle.dcm_mpc_solve_batch_warm(host, threads=8, polished=pol, passes=pas,
                                                         device_batch=B)
    assert (st == 0).all() and pol.all()
    for k, ref in (("status", st), ("iters", it), ("polished", pol), ("passes", pas), ("xi", xi), ("vrp", vrp)):
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref, err_msg=k)


def _handover_batch(oracle, B, horizon, seed):
    """Half the QPs with duplicated facet rows (the polish refuses them: stage 2 solves them)."""
    prob = oracle.assemble_constraints(P.make_batch(B, horizon=horizon, n_footsteps=4, seed=seed))
    for q in range(0, B, 2):
        for k in range(horizon):
            m = prob["nfacets"][q, k]
            c = min(2, 8 - m)
            prob["A"][q, k, m:m + c] = prob["A"][q, k, 0]
            prob["b"][q, k, m:m + c] = prob["b"][q, k, 0]
            prob["nfacets"][q, k] = m + c
    return prob


def test_stage2_list_across_launch_kinds(handle, oracle):
    """The stream's stage-2 list (Handle::stage2_list) through a sequence of solves that take
    every route over it: the cold kernel + IPM list kernel, the fused small-batch kernel (list
    untouched), the warm kernel + IPM list kernel, with fuse_stage2 on and off.  Each solve hands
    QPs over; each equals the oracle bit for bit, so no solve sees a stale count or entry."""
    big = _handover_batch(oracle, 96, 100, 91)
    small = _handover_batch(oracle, 8, 40, 92)
    dbig, dsmall = _to_dev(big), _to_dev(small)

    def check(out, host, **kw):
        torch.cuda.synchronize()
        pol = np.zeros(host["xi_init"].shape[0], np.int32)
        st, xi, vrp, it, lam = oracle.dcm_mpc_solve_batch_warm(host, threads=8, polished=pol, **kw)
        assert not pol.all()   # QPs were handed over
        for k, ref in (("status", st), ("iters", it), ("polished", pol), ("xi", xi), ("vrp", vrp), ("lam", lam)):
            np.testing.assert_array_equal(out[k].cpu().numpy(), ref, err_msg=k)
        return out

    try:
        for fuse in (1, 1, 0, 1):
            native.set_qp_launch_mode(fuse_stage2=fuse)
            cold = check(handle.dcm_mpc_solve(dbig, lambda_out=True), big)
            check(handle.dcm_mpc_solve(dsmall, lambda_out=True), small)
            v, l = cold["vrp"].cpu().numpy().copy(), cold["lam"].cpu().numpy().copy()
            warm = dict(vrp=cold["vrp"], lam=cold["lam"], shift=1, floor=1e-3)
            check(handle.dcm_mpc_solve(dbig, warm=warm, lambda_out=True), big, vrp_ws=v, lam_ws=l, shift=1,
                  floor=1e-3)
    finally:
        native.set_qp_launch_mode(fuse_stage2=1)
