"""Plans with three active contacts (test infrastructure): the contact lists of the reference's own
ContactPhaseList test (src/Planners/tests/ContactPhaseListTest.cpp:32-47, transcribed in
tests/golden/contact_phases.json: left, right and an "additional" contact, phases [4, 5) and
[6, 7) with all three active), turned into batched DCM-MPC plans.

The phases come from the oracle's restatement of ContactPhaseList::createPhases (pinned to the
same fixture by tests/test_oracle.py); each contact is a 0.12 x 0.09 m rectangle, so a phase's
support polygon is the hull of up to 12 corners, listed in std::map order of the list names
(additional, left, right).  poses="identity": every contact at the identity transform, as the
reference test places them (the three rectangles coincide: a 4-facet polygon); "spread": feet
turned out and a hand support ahead, so the three-contact phases have 9-facet hulls (max_facets 16).
"""
import json
import os

import numpy as np

import oracle as O
from blf import problems as P

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
NAMES = ("additional", "left", "right")   # std::map<std::string, ContactList> order


def reference_lists():
    g = json.load(open(os.path.join(GOLDEN, "contact_phases.json")))
    return [[tuple(c) for c in g["lists"][n]] for n in NAMES]


def plan(batch, dt=0.1, knots=75, poses="spread", seed=0, xi_offset=0.01):
    """The plan dict (make_batch's phase-table keys) of `batch` problems over the reference lists;
    knots: length of omega (windows s .. s + N need s + N <= knots); the initial DCM is the first
    phase's centroid plus a uniform offset of up to xi_offset per axis."""
    lists = reference_lists()
    begin, end, active = O.contact_phases(lists)
    NP = len(begin)
    rng = np.random.default_rng(seed)
    corners = np.zeros((batch, NP, 16, 2))
    ncorners = np.zeros((batch, NP), dtype=np.int32)
    for q in range(batch):
        u = rng.uniform(-1.0, 1.0, (3, 4, 3))
        pose = np.zeros((3, 4, 3))      # [list][contact][x, y, yaw]
        if poses == "spread":
            # standing in place, feet turned out, a hand support ahead: a 9-facet hull while all
            # three are in contact (about the most three 0.12 x 0.09 rectangles give)
            for c in range(4):
                pose[1, c] = (0.005 * u[1, c, 0], 0.14 + 0.005 * u[1, c, 1], 1.50 + 0.03 * u[1, c, 2])
                pose[2, c] = (0.005 * u[2, c, 0], -0.14 + 0.005 * u[2, c, 1], -0.03 + 0.03 * u[2, c, 2])
                pose[0, c] = (0.19 + 0.005 * u[0, c, 0], 0.005 * u[0, c, 1], 0.85 + 0.03 * u[0, c, 2])
        for p in range(NP):
            pts = [P.rectangle_corners(pose[l, active[p, l]]) for l in range(3) if active[p, l] >= 0]
            if pts:
                pts = np.concatenate(pts)
                corners[q, p, :len(pts)] = pts
                ncorners[q, p] = len(pts)
    ref = corners.sum(axis=2) / np.maximum(ncorners, 1)[..., None]
    k = np.arange(knots)
    z = 0.53 + 0.01 * np.sin(2.0 * np.pi * k / knots)[None, :] * np.ones((batch, 1))
    omega = np.sqrt(P.GRAVITY / z)
    xi_init = ref[:, 0] + rng.uniform(-xi_offset, xi_offset, (batch, 2))
    return dict(nphases=np.full(batch, NP, dtype=np.int32),
                phase_begin=np.ascontiguousarray(np.broadcast_to(begin, (batch, NP))),
                phase_end=np.ascontiguousarray(np.broadcast_to(end, (batch, NP))),
                phase_corners=corners, phase_ncorners=ncorners, phase_ref=ref,
                omega=np.ascontiguousarray(omega), xi_init=xi_init, dt=dt)
