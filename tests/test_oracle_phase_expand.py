"""Oracle knot -> contact-phase expansion (orc_dcm_phase_expand): the
phase-table path gives exactly the per-knot arrays of the per-knot path (hull of every knot's
corner set), for the first window and for shifted windows of a longer plan.  CPU only."""
import numpy as np

from blf import problems as P


def _oracle_table(oracle, prob, M=8):
    B, NP = prob["phase_ncorners"].shape
    pA = np.zeros((B, NP, M, 2))
    pb = np.zeros((B, NP, M))
    pnf = np.zeros((B, NP), dtype=np.int32)
    for q in range(B):
        for p in range(NP):
            pA[q, p], pb[q, p], pnf[q, p] = oracle.hull2d_hrep(
                prob["phase_corners"][q, p, :prob["phase_ncorners"][q, p]], M)
    return dict(nphases=prob["nphases"], phase_begin=prob["phase_begin"],
                phase_end=prob["phase_end"], phase_A=pA, phase_b=pb, phase_nf=pnf,
                phase_ref=prob["phase_ref"])


def test_phase_table_equals_per_knot_assembly(oracle):
    N, S = 60, 25
    prob = P.make_batch(12, horizon=N + S, n_footsteps=8, seed=17)
    per_knot = oracle.assemble_constraints(prob)
    table = _oracle_table(oracle, prob)
    for s in (0, 1, 9, 10, 24, 25):
        w = P.window(per_knot, s, N)
        ex = oracle.dcm_phase_expand(table, s, prob["dt"], N)
        for k in ("A", "b", "nfacets", "xi_ref", "vrp_ref"):
            np.testing.assert_array_equal(ex[k], w[k], err_msg=f"{k} window {s}")


def test_phase_expand_outside_phases_and_bounds(oracle):
    prob = P.make_batch(3, horizon=40, n_footsteps=4, seed=2)
    table = _oracle_table(oracle, prob)
    table["nphases"] = np.array([0, 2, -5], dtype=np.int32)
    ex = oracle.dcm_phase_expand(table, 0, prob["dt"], 40)
    # problem 0 and 2: no phase at all; problem 1: only the first two phases (to knot 10 + ...)
    assert (ex["nfacets"][0] == -1).all() and (ex["nfacets"][2] == -1).all()
    assert (ex["A"][0] == 0).all() and (ex["xi_ref"][2] == 0).all()
    end1 = table["phase_end"][1, 1]
    t = np.arange(40) * prob["dt"]
    np.testing.assert_array_equal(ex["nfacets"][1] >= 0, t < end1)
    # a window starting past the plan's last phase
    far = oracle.dcm_phase_expand(table, 10 ** 6, prob["dt"], 40)
    assert (far["nfacets"] == -1).all()
