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


def test_c5_two_rank_bench_path_cpu(tmp_path):
    """The config-5 multi-rank path of bench.py, rehearsed on the CPU: two gloo ranks
    launched by torch.distributed.run exactly as the driver launches the scaling bench, each
    running its disjoint robot shard (bench.c5_shard) through the same barriers and
    max-over-ranks timing, with the CPU restatement of the loop (BLF_C5_ORACLE=1) in place of the
    device kernels.  Each rank's robot state after warmup + timed periods equals, bit for bit, the
    same robots' rows of one single-process loop over both shards."""
    import json
    import subprocess
    import sys
    sys.path[:0] = [ROOT, os.path.join(ROOT, "bipedal-locomotion-framework_amd"), os.path.join(ROOT, "oracle")]
    B, N, warmup, steps = 3, 100, 1, 1
    env = dict(os.environ, BLF_C5_ORACLE="1", BLF_BENCH_BACKEND="gloo", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "c5", "--batch", str(B),
           "--horizon", str(N), "--warmup", str(warmup), "--steps", str(steps), "--no-cpu",
           "--dump-state", str(tmp_path)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["batch_per_gpu"] == B and line["state_finite"]
    assert line["qp_status_counts"]["solved"] == 2 * B * steps
    import bench
    import closed_loop as CL
    from blf import closed_loop as DL
    from blf import robot
    model = robot.humanoid24()
    shards = [bench.c5_shard(model, rk, B, N, warmup + steps) for rk in range(2)]
    shared = ("knot_phase", "dt", "schedule")
    plan = {k: (v if k in shared else np.concatenate([s[0][k] for s in shards])) for k, v in shards[0][0].items()}
    st = {k: np.concatenate([s[1][k] for s in shards]) for k in shards[0][1]}
    ref = CL.OracleLoop(model, plan, st, robot.sole_null_poses(model, st), robot.posture_law_arrays(model),
                        DL.CONTACT_PARAMS, horizon=N, compiled=True, threads=2)
    for _ in range(warmup + steps):
        ref.period()
    for rk in range(2):
        got = np.load(os.path.join(tmp_path, f"c5_state_rank{rk}.npz"))
        for k in ref.state:
            np.testing.assert_array_equal(got[k], ref.state[k][rk * B:(rk + 1) * B], err_msg=k)
