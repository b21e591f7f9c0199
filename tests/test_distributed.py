"""World-size-2 test of the sharded path on CPU (gloo): each rank generates and solves its own
shard (the oracle stands in for the device kernel, which needs a GPU), and rank 0 gathers the
solutions with blf.distributed.gather_solutions — the same packing/collective bench.py uses over
RCCL.  The gathered batch must equal a single-process solve of the whole batch bit for bit."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, per_rank, N, q):
    import sys
    sys.path[:0] = [os.path.join(ROOT, "bipedal-locomotion-framework_amd"), os.path.join(ROOT, "oracle")]
    import oracle as O
    from blf import distributed as D
    from blf import problems as P
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = D.shard(per_rank, rank)
    prob = O.assemble_constraints(P.make_batch(count, horizon=N, n_footsteps=4, seed=9, start=start))
    st, xi, vrp, it = O.dcm_mpc_solve_batch(prob, threads=1)
    out = dict(xi=torch.from_numpy(xi), vrp=torch.from_numpy(vrp), status=torch.from_numpy(st),
               iters=torch.from_numpy(it))
    res = D.gather_solutions(out, N, dst=0)
    if rank == 0:
        q.put({k: v.numpy() for k, v in res.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shard_and_gather():
    import sys
    sys.path[:0] = [os.path.join(ROOT, "bipedal-locomotion-framework_amd"), os.path.join(ROOT, "oracle")]
    import oracle as O
    from blf import problems as P
    world, per_rank, N = 2, 6, 30
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per_rank, N, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    full = O.assemble_constraints(P.make_batch(world * per_rank, horizon=N, n_footsteps=4, seed=9))
    st, xi, vrp, it = O.dcm_mpc_solve_batch(full, threads=2)
    np.testing.assert_array_equal(got["xi"], xi)
    np.testing.assert_array_equal(got["vrp"], vrp)
    np.testing.assert_array_equal(got["status"], st)
    np.testing.assert_array_equal(got["iters"], it)
