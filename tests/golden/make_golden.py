"""Generates the committed golden fixtures under tests/golden/ (run in the build container).

Sources (no reference code is executed or copied; the reference is not buildable here, see
DESIGN.md section 6):
  integrator_lti.json   the data of src/System/tests/IntegratorTest.cpp:27-75 (A, B, u, dT, 2 s)
                        run through the oracle; every step is checked against the test's closed
                        form with the test's own tolerance before it is written.
  contact_phases.json   the inputs and the 8 expected phases of
                        src/Planners/tests/ContactPhaseListTest.cpp:15-153, transcribed.
  contact_list.json     src/Planners/tests/ContactListTest.cpp:28-118 present-contact queries.
  hull2d.json           2-D point sets -> Qhull "Qt" facets through scipy.spatial.ConvexHull
                        (scipy bundles Qhull 7.3.2; the reference pins Qhull 8.0.0 — facet order
                        and last bits are not pinned, the facet SET is).
  hull3d_reference.json the 8 points of src/Planners/tests/ConvexHullHelperTest.cpp:15-63 with
                        scipy-Qhull "Qt" facets (documents the 3-D case; the product is 2-D).
  quintic.json          sympy-solved quintic coefficients for random boundary conditions.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def integrator():
    import oracle as O
    A = [[0.0, 1.0], [-2.0, -2.0]]
    B = [[0.0], [2.0]]
    dT = 0.0001
    sim = 2.0
    calls = 0
    while calls < sim / dT:      # `for (int i = 0; i < simulationTime / dT; i++)`
        calls += 1
    x = np.zeros(2)
    checkpoints = []
    for i in range(calls):
        t = dT * i
        closed = np.array([1 - np.exp(-t) * (np.cos(t) + np.sin(t)), 2 * np.exp(-t) * np.sin(t)])
        # Eigen isApprox(b, tol): ||a - b|| <= tol * min(||a||, ||b||)
        assert np.linalg.norm(x - closed) <= 1e-3 * min(np.linalg.norm(x), np.linalg.norm(closed))
        if i % 2500 == 0 or i == calls - 1:
            checkpoints.append([i, float(x[0]), float(x[1])])
        st, x, n = O.lti_euler_integrate(A, B, [1.0], x, 0.0, dT, dT)
        assert st == 0 and n == 1
    return dict(A=A, B=B, u=[1.0], dT=dT, calls=calls, checkpoints=checkpoints,
                final=[float(x[0]), float(x[1])], source="src/System/tests/IntegratorTest.cpp:27-75")


def contact_phases():
    return dict(
        source="src/Planners/tests/ContactPhaseListTest.cpp:15-153",
        lists={"left": [[0.0, 1.0], [2.0, 5.0], [6.0, 7.0]],
               "right": [[0.0, 3.0], [4.0, 7.0]],
               "additional": [[4.0, 5.0], [6.0, 7.5]]},
        # expected phases: begin, end, {list: index of the active contact}
        phases=[[0.0, 1.0, {"left": 0, "right": 0}],
                [1.0, 2.0, {"right": 0}],
                [2.0, 3.0, {"left": 1, "right": 0}],
                [3.0, 4.0, {"left": 1}],
                [4.0, 5.0, {"left": 1, "right": 1, "additional": 0}],
                [5.0, 6.0, {"right": 1}],
                [6.0, 7.0, {"left": 2, "right": 1, "additional": 1}],
                [7.0, 7.5, {"additional": 1}]])


def contact_list():
    return dict(
        source="src/Planners/tests/ContactListTest.cpp:28-118",
        contacts=[[0.1, 0.5], [1.0, 1.5]],
        present=[[1.2, 1], [1.6, 1], [0.6, 0], [0.0, -1]],
        invalid_insertion=[0.9, 1.6],
        touching_insertion=[1.5, 2.0],
        accessor=dict(extra=[[2.0 + i, 2.5 + i] for i in range(49)], size=51))


def hull2d():
    from scipy.spatial import ConvexHull
    rng = np.random.default_rng(2020)
    L, W = 0.12, 0.09

    def rect(x, y, yaw):
        c, s = np.cos(yaw), np.sin(yaw)
        return np.array([[x + c * px - s * py, y + s * px + c * py]
                         for px in (L / 2, -L / 2) for py in (W / 2, -W / 2)])

    sets = [rect(0.0, 0.1, 0.0),                                   # single support, axis aligned
            np.vstack([rect(0.0, 0.1, 0.0), rect(0.0, -0.1, 0.0)]),  # aligned double support
            np.vstack([rect(0.0, 0.1, 0.0), rect(0.2, -0.1, 0.0)]),  # staggered double support
            rect(0.3, -0.1, 0.07)]
    for _ in range(40):
        sets.append(np.vstack([rect(*rng.uniform([-0.1, 0.05, -0.1], [0.3, 0.15, 0.1])),
                               rect(*rng.uniform([-0.1, -0.15, -0.1], [0.3, -0.05, 0.1]))]))
    for n in (3, 5, 7, 9, 12, 16):
        for _ in range(4):
            sets.append(rng.uniform(-1, 1, (n, 2)))
    sets.append(np.array([[np.cos(a), np.sin(a)] for a in np.linspace(0, 2 * np.pi, 12, endpoint=False)]))
    sets.append(np.array([[0, 0], [1, 0], [1, 1], [0, 1], [0.5, 0.5], [0.5, 0], [1, 0.5]], float))
    cases = []
    for p in sets:
        h = ConvexHull(p)          # scipy passes exactly "Qt" for ndim <= 4, like ConvexHullHelper
        eq = h.equations
        cases.append(dict(points=p.tolist(), nfacets=int(len(eq)), A=eq[:, :2].tolist(),
                          b=(-eq[:, 2]).tolist()))
    return dict(source="scipy.spatial.ConvexHull (Qhull 7.3.2, option Qt); reference pins Qhull "
                       "8.0.0 (src/Planners/CMakeLists.txt:22, ConvexHullHelper.cpp:54-58)",
                cases=cases)


def hull3d():
    from scipy.spatial import ConvexHull
    p = np.array([[0.6269, 0.7207, 0.3000], [0.5538, 0.6526, 0.3000], [0.6901, 0.5062, 0.3000],
                  [0.7633, 0.5744, 0.3000], [0.8927, 0.7319, 0.2400], [0.8101, 0.6754, 0.2400],
                  [0.9231, 0.5103, 0.2400], [1.0056, 0.5668, 0.2400]])
    h = ConvexHull(p)
    eq = h.equations
    return dict(source="src/Planners/tests/ConvexHullHelperTest.cpp:15-63", points=p.tolist(),
                A=eq[:, :3].tolist(), b=(-eq[:, 3]).tolist(), outside=[0.0, 0.0, 0.0])


def hull3d_cases():
    """Qhull planes of a few 3-D point sets: the reference test's 8 points, the unit cube (every
    face coplanar: Qhull's "Qt" splits each into two triangles with one plane), a tetrahedron,
    12 points on a sphere, 16 points in a box (some interior)."""
    from scipy.spatial import ConvexHull
    rng = np.random.default_rng(31)
    sph = rng.normal(size=(12, 3))
    sets = [np.array(hull3d()["points"]),
            np.array([[x, y, z] for x in (0.0, 1.0) for y in (0.0, 1.0) for z in (0.0, 1.0)]),
            np.array([[0.0, 0.0, 0.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]),
            sph / np.linalg.norm(sph, axis=1, keepdims=True),
            rng.uniform(-1.0, 2.0, size=(16, 3))]
    cases = []
    for p in sets:
        eq = ConvexHull(p).equations
        cases.append(dict(points=p.tolist(), A=eq[:, :3].tolist(), b=(-eq[:, 3]).tolist()))
    return dict(source="scipy.spatial.ConvexHull (Qhull 7.3.2, Qt always on); reference pins Qhull "
                       "8.0.0 (src/Planners/CMakeLists.txt:22, ConvexHullHelper.cpp:54-58)",
                cases=cases)


def quintic():
    import sympy as sp
    rng = np.random.default_rng(7)
    t = sp.symbols("t")
    c = sp.symbols("c0:6")
    poly = sum(c[i] * t ** i for i in range(6))
    cases = []
    for _ in range(6):
        T = float(rng.uniform(0.2, 1.0))
        bc = rng.uniform(-1, 1, 6)
        eqs = [poly.subs(t, 0) - bc[0], sp.diff(poly, t).subs(t, 0) - bc[1],
               sp.diff(poly, t, 2).subs(t, 0) - bc[2], poly.subs(t, T) - bc[3],
               sp.diff(poly, t).subs(t, T) - bc[4], sp.diff(poly, t, 2).subs(t, T) - bc[5]]
        sol = sp.solve(eqs, c)
        cases.append(dict(T=T, p0=bc[0], v0=bc[1], a0=bc[2], p1=bc[3], v1=bc[4], a1=bc[5],
                          coeffs=[float(sol[ci]) for ci in c]))
    return dict(source="sympy solve of the 6 boundary conditions (quintic Hermite segment)",
                cases=cases)


if __name__ == "__main__":
    for name, fn in [("integrator_lti", integrator), ("contact_phases", contact_phases),
                     ("contact_list", contact_list), ("hull2d", hull2d),
                     ("hull3d_reference", hull3d), ("hull3d", hull3d_cases), ("quintic", quintic)]:
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(fn(), f, indent=1)
        print("wrote", name)
