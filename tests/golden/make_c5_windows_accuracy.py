"""Records, per window of the uncapturable c5 fixtures (c5_failed_windows_r03.npz,
c5_hard_windows.npz), how close the oracle's certified optimum (bit-identical to the device's,
tests/test_gpu_c5_windows.py) comes to the extended-precision solve of the same active set
(qp_reference.lq_solve_ld): max |xi - xi_ld|, max |vrp - vrp_ld| and the largest multiplier, for
the warm solve the closed loop runs and for a cold solve.  tests/test_c5_windows.py checks that
every window stays within its recorded bound; DESIGN.md section 4 (item 9) states them against
north_star's 1e-9.  Run from the repository root:
  python tests/golden/make_c5_windows_accuracy.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "bipedal-locomotion-framework_amd")]
import oracle as O              # noqa: E402
import test_c5_windows as T     # noqa: E402


def errors(prob, xi, vrp):
    import qp_reference
    out = []
    for i in range(prob["omega"].shape[0]):
        A, b, m = prob["A"][i], prob["b"][i], prob["nfacets"][i]
        mask = np.arange(A.shape[1])[None, :] < m[:, None]
        slack = b - np.einsum("kfj,kj->kf", A, vrp[i])
        xl, rl, ll = qp_reference.lq_solve_ld(prob, i, (slack < 1e-9) & mask)
        out.append([float(np.abs(xi[i] - xl).max()), float(np.abs(vrp[i] - rl).max()),
                    float(max(1.0, ll.max()))])
    return out


def main():
    res = {"generator": "tests/golden/make_c5_windows_accuracy.py",
           "columns": ["max |xi - xi_ld|", "max |vrp - vrp_ld|", "max(1, largest multiplier)"]}
    for name in T.FIXTURES:
        prob, d = T.load(name)
        st, xi, vrp, it, lam = T.warm_solve(O, prob, d)
        stc, xic, vrpc, itc = O.dcm_mpc_solve_batch(prob, threads=8, device_batch=16384)
        res[name] = {"warm": errors(prob, xi, vrp), "cold": errors(prob, xic, vrpc)}
    with open(os.path.join(HERE, "c5_windows_accuracy.json"), "w") as f:
        json.dump(res, f, indent=0)


if __name__ == "__main__":
    main()
