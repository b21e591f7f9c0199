"""CPU tests of the synthetic workload generator (blf.problems) and its agreement with the
oracle's restatement of ContactPhaseList."""
import numpy as np

import oracle as O
from blf import problems as P


def test_shards_are_reproducible():
    full = P.make_batch(12, horizon=40, seed=5)
    part = P.make_batch(4, horizon=40, seed=5, start=8)
    for k in ("xi_init", "omega", "xi_ref", "vrp_ref", "corners", "ncorners"):
        np.testing.assert_array_equal(full[k][8:], part[k])


def test_every_knot_has_a_support_polygon():
    for F, N in ((2, 1), (4, 50), (6, 100), (8, 130)):
        prob = P.make_batch(3, horizon=N, n_footsteps=F, seed=1)
        assert set(np.unique(prob["ncorners"])) <= {4, 8}
        assert (prob["omega"] > 0).all()
        A, b, m = O.hull2d_hrep(prob["corners"][0, 0, :prob["ncorners"][0, 0]], 8)
        assert m >= 4
        # the reference VRP (centroid) is strictly inside its polygon
        assert (A[:m] @ prob["vrp_ref"][0, 0] < b[:m]).all()


def test_knot_times_fall_on_contact_events_exactly():
    sched = P.contact_schedule(6, 100)
    dt = 0.02
    phases = P.phases_from_schedule(sched, dt)
    # contact times are knot * dt, so each phase boundary is one of the knot times
    knots = {k * dt for k in range(200)}
    for b0, e0, _ in phases[:-1]:
        assert b0 in knots and e0 in knots


def test_swing_splines_shapes():
    prob = P.make_batch(5, horizon=100, n_footsteps=6, seed=2)
    kt, kp, tq = P.swing_splines(prob, queries=16)
    assert kt.shape[1] == 3 and kp.shape[1:] == (3, 3, 3) and tq.shape[1] == 16
    assert (np.diff(kt, axis=1) > 0).all()
