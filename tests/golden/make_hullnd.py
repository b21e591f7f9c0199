"""Writes tests/golden/hullnd.json: n x p point sets and the supporting hyperplanes Qhull gives for
them (scipy.spatial.ConvexHull = Qhull, the library ConvexHullHelper.cpp:35-99 hands its n x p
matrix to), deduplicated to one row per plane (Qhull "Qt" emits one row per simplex of a split
facet).  Run from the repo root: python tests/golden/make_hullnd.py"""
import itertools
import json
import os

import numpy as np
from scipy.spatial import ConvexHull


def qhull_planes(P):
    if P.shape[1] == 1:
        return [([1.0], float(P.max())), ([-1.0], float(-P.min()))]
    out = []
    for e in ConvexHull(P).equations:   # a . x + off <= 0 inside
        a, b = e[:-1], -e[-1]
        if not any(np.allclose(a, x, atol=1e-9) and abs(b - y) < 1e-9 for x, y in out):
            out.append((a.tolist(), float(b)))
    return out


def main():
    rng = np.random.default_rng(2024)
    sets = []
    for dim in range(1, 8):
        for p in (dim + 1, dim + 4, min(dim + 8, 14)):
            sets.append((f"gaussian d{dim} p{p}", rng.normal(size=(p, dim))))
    sets.append(("hypercube d4", np.array(list(itertools.product([0.0, 1.0], repeat=4)))))
    sets.append(("hypercube d5 (32 points)", np.array(list(itertools.product([-1.0, 2.0], repeat=5)))))
    cross = np.concatenate([np.eye(6), -np.eye(6)]) * 1.5
    sets.append(("cross-polytope d6", cross))
    sph = rng.normal(size=(20, 4))
    sets.append(("sphere d4 p20", sph / np.linalg.norm(sph, axis=1, keepdims=True)))
    box = np.array(list(itertools.product([0.0, 1.0], repeat=3)))
    sets.append(("cube d3 + interior points (20)", np.concatenate([box, rng.uniform(0.1, 0.9, (12, 3))])))
    sets.append(("simplex d8", np.concatenate([np.zeros((1, 8)), np.eye(8)])))
    out = [dict(name=n, points=P.tolist(), planes=[dict(a=a, b=b) for a, b in qhull_planes(P)]) for n, P in sets]
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "hullnd.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=None)
    print(f"wrote {path}: {len(out)} point sets")


if __name__ == "__main__":
    main()
