"""GPU parity of the knot -> contact-phase expansion (blf_dcm_phase_expand) against the oracle
(orc_dcm_phase_expand), bit for bit, and the end-to-end receding-horizon input path: phase
polygons built once on the device, expanded per window, solved — identical to the per-knot hull
path."""
import numpy as np
import pytest
import torch

from blf import problems as P
from test_oracle_phase_expand import _oracle_table

pytestmark = pytest.mark.gpu
TABLE_KEYS = ("nphases", "phase_begin", "phase_end", "phase_A", "phase_b", "phase_nf", "phase_ref")


def _dev(d, keys):
    return {k: torch.from_numpy(np.ascontiguousarray(d[k])).cuda() for k in keys}


@pytest.mark.parametrize("N,S,B", [(100, 20, 64), (37, 3, 5), (250, 1, 16)])
def test_phase_expand_bitwise(handle, oracle, N, S, B):
    prob = P.make_batch(B, horizon=N + S, n_footsteps=8, seed=29)
    table = _oracle_table(oracle, prob)
    dtab = _dev(table, TABLE_KEYS)
    for s in range(0, S + 1, max(1, S // 4)):
        ex = oracle.dcm_phase_expand(table, s, prob["dt"], N)
        out = handle.dcm_phase_expand(dtab, s, prob["dt"], N)
        torch.cuda.synchronize()
        for k in ("A", "b", "nfacets", "xi_ref", "vrp_ref"):
            np.testing.assert_array_equal(out[k].cpu().numpy(), ex[k], err_msg=k)


def test_phase_expand_edge_cases(handle, oracle):
    prob = P.make_batch(6, horizon=30, n_footsteps=4, seed=2)
    table = _oracle_table(oracle, prob, M=6)
    table["nphases"] = np.array([0, 2, -5, 99, 1, 3], dtype=np.int32)
    table["phase_begin"] = table["phase_begin"].copy()
    table["phase_begin"][4, 0] = np.nan                       # never <= t
    dtab = _dev(table, TABLE_KEYS)
    for start in (0, 7, 10 ** 6):
        ex = oracle.dcm_phase_expand(table, start, prob["dt"], 30)
        out = handle.dcm_phase_expand(dtab, start, prob["dt"], 30)
        torch.cuda.synchronize()
        for k in ("A", "b", "nfacets", "xi_ref", "vrp_ref"):
            np.testing.assert_array_equal(out[k].cpu().numpy(), ex[k], err_msg=k)


def test_phase_table_path_equals_per_knot_path(handle, oracle):
    """Device hull over the phases + expansion + QP == device hull over every knot + QP."""
    N, S, B = 100, 12, 128
    prob = P.make_batch(B, horizon=N + S, n_footsteps=8, seed=31)
    ptab = handle.phase_table(
        torch.from_numpy(prob["nphases"]).cuda(), torch.from_numpy(prob["phase_begin"]).cuda(),
        torch.from_numpy(prob["phase_end"]).cuda(), torch.from_numpy(prob["phase_corners"]).cuda(),
        torch.from_numpy(prob["phase_ncorners"]).cuda(),
        ref=torch.from_numpy(prob["phase_ref"]).cuda())
    A, b, nf = handle.assemble_constraints(torch.from_numpy(prob["corners"]).cuda(),
                                           torch.from_numpy(prob["ncorners"]).cuda())
    per_knot = dict(xi_init=prob["xi_init"], omega=prob["omega"], xi_ref=prob["xi_ref"],
                    vrp_ref=prob["vrp_ref"], A=A.cpu().numpy(), b=b.cpu().numpy(),
                    nfacets=nf.cpu().numpy())
    for s in (0, 5, S):
        w = P.window(per_knot, s, N)
        ex = handle.dcm_phase_expand(ptab, s, prob["dt"], N)
        for k in ("A", "b", "nfacets", "xi_ref", "vrp_ref"):
            np.testing.assert_array_equal(ex[k].cpu().numpy(), w[k], err_msg=f"{k} window {s}")
        dev = dict(ex, xi_init=torch.from_numpy(w["xi_init"]).cuda(),
                   omega=torch.from_numpy(w["omega"]).cuda())
        out = handle.dcm_mpc_solve(dev)
        ref = handle.dcm_mpc_solve(_dev(w, ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b",
                                            "nfacets")))
        torch.cuda.synchronize()
        assert torch.equal(out["vrp"], ref["vrp"]) and torch.equal(out["xi"], ref["xi"])
        if s == 0:   # later windows keep the plan's xi_init: harder QPs, some hit the cap
            assert (out["status"] == 0).all()
        assert torch.equal(out["status"], ref["status"]) and torch.equal(out["iters"], ref["iters"])
