"""The multi-GPU bench path's collectives over RCCL on the device.

A one-GPU box cannot hold two RCCL ranks (RCCL refuses two ranks on one device), so this runs the
exact calls bench.py makes on every rank -- init_process_group("nccl", device_id=...), the
device-tensor all_reduce(MAX) of the step time, blf.distributed.gather_solutions of the solved
shard's device tensors -- in a world of one, in a child process (its own process group and HIP
context).  The gathered rows must be the shard's solution bit for bit, and the shard (generated at
a nonzero global offset) must match the oracle.  The world-size-2 exchange itself is covered on
CPU by tests/test_distributed.py (gloo)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(port, B, N, start, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "bipedal-locomotion-framework_amd")]
    import torch.distributed as dist
    from blf import distributed as D
    from blf import native, problems as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        h = native.Handle(0)
        prob = P.make_batch(B, horizon=N, n_footsteps=6, seed=P.SEED, start=start)
        d = {k: torch.from_numpy(prob[k]).to(dev) for k in ("xi_init", "omega", "xi_ref", "vrp_ref")}
        A, b, nf = h.assemble_constraints(torch.from_numpy(prob["corners"]).to(dev),
                                          torch.from_numpy(prob["ncorners"]).to(dev))
        d.update(A=A, b=b, nfacets=nf)
        out = h.dcm_mpc_solve(d)
        t = torch.tensor([1.25], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        got = D.gather_solutions(out, N, dst=0)
        torch.cuda.synchronize()
        q.put(dict(tmax=float(t.item()), on_device=all(v.is_cuda for v in got.values()),
                   got={k: v.cpu().numpy() for k, v in got.items()},
                   direct={k: out[k].cpu().numpy() for k in ("xi", "vrp", "status", "iters")},
                   host={k: np.ascontiguousarray(v.cpu().numpy()) for k, v in
                         (("A", A), ("b", b), ("nfacets", nf))} |
                        {k: prob[k] for k in ("xi_init", "omega", "xi_ref", "vrp_ref")}))
    finally:
        dist.destroy_process_group()


def test_rccl_gather_of_device_shard(oracle):
    B, N, start = 96, 100, 5 * 32768
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), B, N, start, q))
    p.start()
    res = q.get(timeout=100)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert res["tmax"] == 1.25 and res["on_device"]
    for k in ("xi", "vrp", "status", "iters"):
        np.testing.assert_array_equal(res["got"][k], res["direct"][k], err_msg=k)
    st, xi, vrp, it = oracle.dcm_mpc_solve_batch(res["host"], threads=4)
    np.testing.assert_array_equal(res["got"]["xi"], xi)
    np.testing.assert_array_equal(res["got"]["vrp"], vrp)
    np.testing.assert_array_equal(res["got"]["iters"], it)
    assert (res["got"]["status"] == 0).all() and (np.asarray(st) == 0).all()
