"""ConvexHullHelper on n x p points in any dimension (ConvexHullHelper.cpp:35-99 hands the n x p
matrix to Qhull): the oracle (orc_hullnd_hrep) against Qhull's planes (tests/golden/hullnd.json,
written by tests/golden/make_hullnd.py with scipy's Qhull), and the device kernel
(blf_hullnd_hrep, one wavefront per set) bit for bit against the oracle."""
import itertools
import json
import os

import numpy as np
import pytest

import oracle as O

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _golden():
    with open(os.path.join(GOLDEN, "hullnd.json")) as f:
        return json.load(f)


def _same_planes(A, b, m, planes):
    if m != len(planes):
        return False
    for pl in planes:
        a = np.asarray(pl["a"])
        if not any(np.allclose(A[i], a, atol=1e-9) and abs(b[i] - pl["b"]) < 1e-9 for i in range(m)):
            return False
    return True


@pytest.mark.parametrize("case", range(len(_golden())))
def test_oracle_hullnd_matches_qhull(case):
    g = _golden()[case]
    P = np.asarray(g["points"])
    A, b, m = O.hullnd_hrep(P, max_facets=1024)
    assert _same_planes(A, b, m, g["planes"]), g["name"]
    for q in P:   # every input point passes doesPointBelongToConvexHull exactly (b is the max)
        assert O.halfspace_contains(A[:m], b[:m], m, q)


def test_oracle_hullnd_degenerate_and_overflow():
    rng = np.random.default_rng(3)
    flat = rng.normal(size=(12, 4))
    flat[:, 2] = 0.25                       # spans 3 of 4 dimensions
    assert O.hullnd_hrep(flat, 64)[2] == -1
    assert O.hullnd_hrep(rng.normal(size=(4, 4)), 64)[2] == -1       # fewer than dim + 1 points
    cube = np.array(list(itertools.product([0.0, 1.0], repeat=4)))
    A, b, m = O.hullnd_hrep(cube, 7)        # 8 facets do not fit in 7 rows
    assert m == -1 and not A.any() and not b.any()
    assert O.hullnd_hrep(np.ones((3, 1)), 4)[2] == -1                 # 1-D, one distinct point


def _pack(sets, P):
    D = sets[0].shape[1]
    pts = np.zeros((len(sets), P, D))
    n = np.zeros(len(sets), dtype=np.int32)
    for i, s in enumerate(sets):
        pts[i, : len(s)] = s
        n[i] = len(s)
    return pts, n


@pytest.mark.gpu
@pytest.mark.parametrize("dim", range(1, 9))
def test_gpu_hullnd_bitwise(handle, dim):
    """Ragged point sets of one dimension (golden sets of that dimension, random sets, a flat set,
    too few points, facet overflow): rows, offsets and counts bit for bit the oracle's."""
    import torch
    rng = np.random.default_rng(100 + dim)
    sets = [np.asarray(g["points"]) for g in _golden() if len(g["points"][0]) == dim and len(g["points"]) <= 32]
    for p in (dim + 1, dim + 3, min(dim + 9, 16)):
        sets.append(rng.normal(size=(p, dim)))
        sets.append(np.round(rng.uniform(-2, 2, size=(p, dim)) * 2) / 2)   # lattice: coplanar facets
    flat = rng.normal(size=(dim + 5, dim))
    flat[:, -1] = 0.5
    sets += [flat, rng.normal(size=(dim, dim))]
    P = max(len(s) for s in sets)
    pts, n = _pack(sets, P)
    for M in (1024, dim + 2):
        A, b, nf = handle.hullnd_hrep(torch.from_numpy(pts).cuda(), torch.from_numpy(n).cuda(), max_facets=M)
        A, b, nf = A.cpu().numpy(), b.cpu().numpy(), nf.cpu().numpy()
        for i, s in enumerate(sets):
            Ao, bo, mo = O.hullnd_hrep(s, M)
            assert nf[i] == mo, (i, M)
            np.testing.assert_array_equal(A[i], Ao)
            np.testing.assert_array_equal(b[i], bo)


@pytest.mark.gpu
def test_gpu_hullnd_matches_qhull_and_contains(handle):
    """Every golden set through the device, as sets of planes against Qhull; the points pass
    blf_halfspace_contains, a point pushed past each facet fails."""
    import torch
    for g in _golden():
        P = np.asarray(g["points"])
        if len(P) > 32:
            continue
        A, b, nf = handle.hullnd_hrep(torch.from_numpy(P[None]).cuda(),
                                      torch.tensor([len(P)], dtype=torch.int32).cuda(), max_facets=1024)
        A, b, m = A.cpu().numpy()[0], b.cpu().numpy()[0], int(nf[0])
        assert _same_planes(A, b, m, g["planes"]), g["name"]
        out = np.array([P[np.argmax(P @ A[i])] + 0.1 * A[i] for i in range(m)])   # past facet i
        q = np.concatenate([P, out])
        inside = handle.halfspace_contains(torch.from_numpy(np.repeat(A[None], len(q), 0)).cuda(),
                                           torch.from_numpy(np.repeat(b[None], len(q), 0)).cuda(),
                                           torch.full((len(q),), m, dtype=torch.int32).cuda(),
                                           torch.from_numpy(q).cuda()).cpu().numpy()
        assert inside[: len(P)].all() and not inside[len(P):].any(), g["name"]


@pytest.mark.gpu
def test_gpu_hullnd_argument_errors(handle):
    import torch
    from blf import native
    pts = torch.zeros((1, 33, 4), dtype=torch.float64).cuda()
    n = torch.tensor([5], dtype=torch.int32).cuda()
    with pytest.raises(native.BlfError):   # more than BLF_HULLND_MAX_POINTS
        handle.hullnd_hrep(pts, n)
    with pytest.raises(native.BlfError):   # dim 9
        handle.hullnd_hrep(torch.zeros((1, 10, 9), dtype=torch.float64).cuda(), n)
    with pytest.raises(native.BlfError):   # C(32, 8) subsets above the cap
        handle.hullnd_hrep(torch.zeros((1, 32, 8), dtype=torch.float64).cuda(), n)
