"""Benchmark: DCM-MPC QP solves/sec (batch, horizon 100) on 1..8 MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): per GPU, a batch of 4096 horizon-100 time-varying DCM MPC
QPs (6-footstep plans, M = 8 facet slots, fp64), inputs resident in HBM.  One step = one
blf_dcm_mpc_solve over the whole per-GPU batch (every QP solved from a cold start to
tol_mu 1e-16).  Multi-GPU: one process per GPU (torch.distributed.run), each rank solves its own
shard of independent problems — no data-path collective (scaling "weak"); the RCCL gather of the
solutions to rank 0 is timed separately and reported as gather_ms.

Prints ONE JSON line on rank 0 (the driver's contract), with two extra objects:
  roofline      HBM roofline of the dominant kernel (dcm_mpc_cold_kernel: the fp32 active-set
                search and the fp64 certified passes), from the algorithmic bytes per QP
                 and the kernel's average duration measured with HIP events
                on the launch stream; plus the executed fp64 fraction and the VALU issue fraction
                (the roof that binds this kernel).
  cpu_baseline  the CPU oracle (same algorithm, C, gcc -O3, one problem per thread)
                on every CPU this process may use (affinity set capped by the cgroup CPU quota),
                rank 0 only, on a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "bipedal-locomotion-framework_amd"))

HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6    # MI355X fp64 vector (spec)


def algorithmic_bytes_per_qp(N, M):
    f64 = 2 + N + 2 * (N + 1) + 2 * N + 2 * N * M + N * M + 2 * (N + 1) + 2 * N
    i32 = N + 2
    return 8 * f64 + 4 * i32


def profiled_summary():
    """The newest committed rocprofv3 summary of the dominant kernel (profiles/*_summary.json,
    written by tools/summarize_profile.py from separate FETCH_SIZE / WRITE_SIZE / SQ passes) whose
    recorded build is the library this process loaded (lib_src_hash equal to
    native.build_provenance()'s); bench.py cannot read PMC counters itself.  Counters of another
    build describe other code, so without a match the counter-derived fields are null.
    Returns (summary, path) or (None, None)."""
    import glob
    import re
    from blf import native
    lib_hash = native.build_provenance().get("lib_src_hash")
    # newest by name (profiles/rNN_vMM_<tag>_summary.json; file times do not survive the copy to a
    # box), numbers compared as numbers so v10 sorts after v9
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_summary.json")),
                   key=lambda f: [int(t) if t.isdigit() else t
                                  for t in re.split(r"(\d+)", os.path.basename(f))])
    for path in reversed(files):
        with open(path) as f:
            s = json.load(f)
        if "dcm_mpc_" not in s.get("dominant_kernel", ""):   # the QP kernels (cold / warm / ipm)
            continue
        if lib_hash and (s.get("build") or {}).get("lib_src_hash") == lib_hash:
            return s, os.path.relpath(path, ROOT)
    return None, None


def profiled_traffic():
    """HBM bytes per launch of the dominant kernel (corrected FETCH + WRITE), or None."""
    s, path = profiled_summary()
    t = s.get("hbm_traffic_per_launch") if s else None
    if not t:
        return None, None
    return t["total_bytes_corrected"], path


SIMDS, CLOCK_HZ = 1024, 2.4e9
F64_CYCLES, VALU32_CYCLES = 4, 2   # wave64 on a SIMD-32: fp64 at 16 lanes / cycle, 32-bit at 32


def valu_issue(kernel_ms):
    """The roof that binds the QP kernel: VALU issue.  VALU wave-instructions per launch from the
    committed SQ_INSTS_VALU pass (fp64 FMA / MUL / ADD counted at 4 SIMD cycles, every other VALU
    instruction at 2), over the chip's SIMD cycles in the kernel time measured here (1024 SIMDs at
    the 2.4 GHz peak clock)."""
    s, path = profiled_summary()
    v = s.get("valu_issue") if s else None
    if not v:
        return None
    n = v["valu_insts_per_launch"]
    f = v.get("fp64_insts_per_launch")
    n64 = (f["fma"] + f["mul"] + f["add"]) if f else n
    cycles = F64_CYCLES * n64 + VALU32_CYCLES * (n - n64)
    return {"valu_insts_per_launch": n, "fp64_insts_per_launch": n64,
            "frac": cycles / (SIMDS * CLOCK_HZ * kernel_ms * 1e-3),
            "source": path}


FP64_PEAK_TFLOPS = 78.6   # MI355X vector fp64 (MI355X_MICROARCH.md)


def fbd_sq_summary():
    """The newest committed SQ summary of fbd_euler_kernel (profiles/*_fbd_euler_sq.json, written by
    tools/sq_summary.py from tools/gpu_sq.sh's passes with SQ_EXTRA=1) recorded on the library this
    process loaded; (None, None) without a match."""
    import glob
    import re
    from blf import native
    lib_hash = native.build_provenance().get("lib_src_hash")
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_fbd_euler_sq.json")),
                   key=lambda f: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(f))])
    for path in reversed(files):
        with open(path) as f:
            s = json.load(f)
        if lib_hash and (s.get("build") or {}).get("lib_src_hash") == lib_hash:
            return s, os.path.relpath(path, ROOT)
    return None, None


def fbd_roofline(kernel_ms, robots_per_launch):
    """configs[4]'s dominant kernel, fbd_euler_kernel (one control period of the dynamics of a group
    of robots per launch): fp64 FLOP/s against the vector fp64 peak.  flops per launch = the executed
    fp64 lanes of the hash-matched SQ pass, 64 x (2 FMA + MUL + ADD) wave-instructions (FMA counted
    twice; transcendental and conversion instructions not counted); kernel_ms = the launches' mean
    duration from HIP events on their own streams in the timed region."""
    s, path = fbd_sq_summary()
    med = s["median_per_dispatch"] if s else None
    flops = None
    if med and "SQ_INSTS_VALU_FMA_F64" in med:
        flops = 64.0 * (2.0 * med["SQ_INSTS_VALU_FMA_F64"] + med["SQ_INSTS_VALU_MUL_F64"]
                        + med["SQ_INSTS_VALU_ADD_F64"])
    achieved = flops / (kernel_ms * 1e-3) / 1e12 if flops else None
    wc = med.get("SQ_WAVE_CYCLES") if med else None
    return {"bound": "fp64", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
            "frac": achieved / FP64_PEAK_TFLOPS if achieved else None, "traffic": None,
            "kernel": "fbd_euler_kernel (one period: 19 ForwardEuler steps of the 30-DoF dynamics)",
            "kernel_ms": kernel_ms, "robots_per_launch": robots_per_launch,
            "fp64_flops_per_launch": flops,
            "wait_inst_lds_frac": (med["SQ_WAIT_INST_LDS"] / wc) if med and wc and "SQ_WAIT_INST_LDS" in med else None,
            "traffic_source": path}


def cpu_baseline(host, N, seconds, threads):
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    B = host["omega"].shape[0]
    # the CPU-efficient form of the same algorithm: sequential recursions instead of the device's
    # lane scans (oracle `sequential` mode; identical iterates up to rounding)
    prm = O.default_params(N, max_facets=host["b"].shape[2], sequential=1)
    O.dcm_mpc_solve_batch(host, params=prm, threads=threads, count=min(B, 64))   # warm-up
    solved, t0 = 0, time.perf_counter()
    while True:
        st, _, _, _ = O.dcm_mpc_solve_batch(host, params=prm, threads=threads)
        solved += B
        el = time.perf_counter() - t0
        if el >= seconds:
            break
    assert (st == 0).all()
    # single-problem latency (one thread), BASELINE.md C1-style figure at this horizon
    t1 = time.perf_counter()
    for i in range(20):
        O.dcm_mpc_solve(host, params=prm, index=i)
    lat_us = (time.perf_counter() - t1) / 20 * 1e6
    return dict(value=solved / el, unit="QP/s", cores=threads, kind="port",
                sample=f"{solved} solves = {solved // B} passes over the same {B} horizon-{N} QPs "
                       f"in {el:.2f} s wall on {threads} threads (oracle/blf_oracle.c sequential "
                       f"mode, gcc -O3 -mfma, one problem per thread)",
                single_thread_latency_us=round(lat_us, 1), **host_cpu_info())


def cpu_threads():
    """The CPUs this process can actually run on: the affinity set, capped by the cgroup CPU quota
    when there is one (a GPU box shows the whole machine in its affinity set, 256 CPUs, but grants
    one GPU's process a quota of 16; more threads than the quota only time-slice)."""
    info = host_cpu_info()
    n = info["affinity_cpus"]
    if info["cgroup_cpu_quota"]:
        n = min(n, max(1, int(info["cgroup_cpu_quota"])))
    return n


def host_cpu_info():
    """What the host offers this process: the affinity set, the cgroup CPU quota (if any) and
    os.cpu_count(); the CPU baseline runs one thread per CPU of the affinity set."""
    info = {"affinity_cpus": len(os.sched_getaffinity(0)), "os_cpu_count": os.cpu_count()}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        info["cgroup_cpu_quota"] = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        info["cgroup_cpu_quota"] = None
    return info


def emit(line):
    """Print one JSON result line with the build provenance of the library it measured: the source
    hash compiled into lib/libblf.so (blf_version) against the hash of this tree's sources."""
    from blf import native
    line["build"] = native.build_provenance()
    print(json.dumps(line), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=4096, help="QPs per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None,
                    help="QPs over all GPUs, split into contiguous per-rank shards (strong scaling; "
                         "configs[3] is --global-batch 262144 on 8 GPUs)")
    ap.add_argument("--horizon", type=int, default=100)
    ap.add_argument("--cpu-seconds", type=float, default=5.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--dump-state", default=None,
                    help="c5: write each rank's final robot state to DIR/c5_state_rank<r>.npz")
    ap.add_argument("--c5-groups", type=int, default=2,
                    help="c5: robots in this many groups, each closed loop on its own stream "
                         "(round 4, profiles/r04_v2_c5_g*.log: 1 group 5.88 / 5.88 ms, 2 groups "
                         "5.74 / 5.67 ms per period; 3 groups 6.05 / 6.13 ms, profiles/r04f_*)")
    ap.add_argument("--tol-polish", type=float, default=None,
                    help="override blf_dcm_mpc_default_params' tol_polish (also the CPU baseline's)")
    ap.add_argument("--expand-path", action="store_true",
                    help="rh / c3 / c5: expand the window through HBM (blf_dcm_phase_expand) and "
                         "solve it (the two calls blf_dcm_mpc_solve_phased fuses; A/B only)")
    ap.add_argument("--workload", choices=("c1", "c2", "c3", "c5", "rh", "mc"), default="c2",
                    help="c2 (default, the driver's metric): configs[1]; c1: configs[0] single-solve "
                         "latency (4 footsteps, N=50) on the GPU and the CPU; c3: configs[2] pipeline "
                         "(hull H-rep + QP + swing splines, B=65536); c5: configs[4] closed loop "
                         "(robot DCM -> warm-started QP -> joint references -> 30-DoF floating-"
                         "base dynamics with contact feet, B=16384 per GPU, multi-rank); rh: "
                         "receding-horizon advance() (phase expansion + warm-started QP, B=4096); "
                         "mc: plans with three-contact phases (the reference ContactPhaseList "
                         "test's lists, 16 facet slots, N=50): cold solves and warm windows")
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        # checked before any HIP call: a scaling run launched without torch.distributed.run would
        # otherwise measure one GPU and report it as n_gpus = 1
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}; launch N > 1 with "
                 f"python -m torch.distributed.run --nproc-per-node N bench.py --gpus N")
    if args.workload not in ("c2", "c5") and world > 1:
        sys.exit(f"bench.py: --workload {args.workload} runs on one GPU")
    if args.workload != "c2":
        return other_workload(args)

    import numpy as np
    import torch
    import torch.distributed as dist
    from blf import native
    from blf import problems as P

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.global_batch is not None:
        if args.global_batch % world:
            sys.exit(f"bench.py: --global-batch {args.global_batch} is not divisible by {world} ranks")
        args.batch = args.global_batch // world
    # RCCL (backend "nccl") over xGMI on a node; BLF_BENCH_BACKEND=gloo rehearses the multi-rank
    # path on a single GPU (every rank then shares device LOCAL_RANK % device_count)
    backend = os.environ.get("BLF_BENCH_BACKEND", "nccl")
    local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    h = native.Handle(local)

    B, N = args.batch, args.horizon
    prob = P.make_batch(B, horizon=N, n_footsteps=6, seed=P.SEED, start=rank * B)
    d = {k: torch.from_numpy(prob[k]).to(dev) for k in ("xi_init", "omega", "xi_ref", "vrp_ref")}
    A, b, nf = h.assemble_constraints(torch.from_numpy(prob["corners"]).to(dev),
                                      torch.from_numpy(prob["ncorners"]).to(dev))
    d.update(A=A, b=b, nfacets=nf)
    M = b.shape[2]
    params = native.default_params(N, max_facets=M)
    out = h.dcm_mpc_solve(d, params)
    torch.cuda.synchronize()
    assert int((out["status"] != 0).sum()) == 0, "unsolved QPs in the bench batch"

    stream = torch.cuda.current_stream()
    for _ in range(args.warmup):
        h.dcm_mpc_solve(d, params, out=out)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        h.dcm_mpc_solve(d, params, out=out)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps      # one launch per step on this stream
    if world > 1:
        t = torch.tensor([elapsed], device=dev if backend == "nccl" else "cpu",
                         dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    iters = out["iters"].to(torch.int64)
    polished = out["polished"].to(torch.float64)

    # RCCL gather of every rank's solutions to rank 0 (timed separately, not in `value`)
    gather_ms = None
    if world > 1:
        from blf import distributed as D
        dist.barrier()
        torch.cuda.synchronize()
        tg = time.perf_counter()
        D.gather_solutions(out if backend == "nccl" else {k: v.cpu() for k, v in out.items()},
                           N, dst=0)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - tg) * 1e3

    if rank == 0:
        total = world * B * args.steps
        bpq = algorithmic_bytes_per_qp(N, M)
        achieved = bpq * B / (kernel_ms * 1e-3) / 1e9
        traffic, traffic_src = profiled_traffic()
        # executed fp64 flops of the dominant kernel's launch from the committed SQ pass (FMA
        # counts two, 64 lanes per wave instruction, masked lanes included): the active-set
        # passes' scans with their Kogge-Stone redundancy, i.e. what the SIMDs actually did
        pmc, _ = profiled_summary()
        f64 = ((pmc or {}).get("valu_issue") or {}).get("fp64_insts_per_launch")
        fp64_exec_tf = (64.0 * (2.0 * f64["fma"] + f64["mul"] + f64["add"]) / (kernel_ms * 1e-3)
                        / 1e12) if f64 else None
        vi = valu_issue(kernel_ms)
        line = {
            "metric": "DCM-MPC QP solves/sec (batch, horizon=100) at 1/2/4/8 MI355X",
            "value": total / elapsed,
            "unit": "QP/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.global_batch is None else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "arith": "fp32 active-set search, fp64 certified equality-constrained solve (the "
                     "returned optimum is fp64)",
            "data": "synthetic (6-footstep plans, SeedSequence-keyed Philox per problem)",
            "config": {"workload": (f"configs[1]: batch={B} DCM-MPC QPs per GPU, horizon={N}, "
                                    f"M={M} facet slots, fp64, one wavefront per QP"
                                    if args.global_batch is None else
                                    f"configs[3]-style: global batch {args.global_batch} "
                                    f"DCM-MPC QPs over {world} GPUs ({B} per rank), horizon={N}"),
                       "batch_per_gpu": B, "global_batch": B * world, "horizon": N,
                       "max_facets": M,
                       "parallelism": f"shard{world} (independent problems)"},
            # "bound": the roof that binds the kernel as measured (VALU issue and latency,
            # DESIGN.md 3.1), not HBM; achieved / peak / frac stay the HBM stream the contract
            # prices (algorithmic bytes over the kernel time against 8 TB/s)
            "roofline": {"bound": "valu_issue", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": "dcm_mpc_cold_kernel<2> (fp32 active-set search + fp64 "
                                   "certified passes; + the IPM kernel's stage 2 on the QPs it hands "
                                   "over, inside the same event pair)",
                         "kernel_ms": kernel_ms,
                         "bytes_per_qp": bpq,
                         # what binds this kernel is neither HBM nor MFMA: VALU issue and the
                         # latency of the scans' lane-shuffle chains
                         "binding_roof": {"kind": "valu_issue",
                                          "frac": vi["frac"] if vi else None},
                         "valu_issue": vi,
                         "fp64_valu": {"executed_tflops": fp64_exec_tf,
                                       "peak_tflops": FP64_PEAK_TFLOPS,
                                       "executed_frac": (fp64_exec_tf / FP64_PEAK_TFLOPS
                                                         if fp64_exec_tf else None)},
                         "mean_ipm_iters": float(iters.float().mean()),
                         "polished_frac": float(polished.mean())},
            "gather_ms": gather_ms,
        }
        if not args.no_cpu:
            threads = cpu_threads()
            host = dict(prob, A=A.cpu().numpy(), b=b.cpu().numpy(), nfacets=nf.cpu().numpy())
            line["cpu_baseline"] = cpu_baseline(host, N, args.cpu_seconds, threads)
        emit(line)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _timed(fn, steps, warmup):
    import torch
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def other_workload(args):
    """Secondary single-GPU measurements of BASELINE configs[2] and configs[4] (not the driver's
    headline line; DESIGN.md section 9 records them)."""
    import numpy as np
    import torch
    from blf import native
    from blf import problems as P
    from blf import robot
    if args.workload == "c5":
        return closed_loop(args)
    h = native.Handle(0)
    dev = torch.device("cuda", 0)
    N = args.horizon
    if args.workload == "rh":
        return receding_horizon(args, h, dev)
    if args.workload == "mc":
        return three_contact(args, h, dev)
    if args.workload == "c1":
        return single_solve_latency(args, h, dev)
    if args.workload == "c3":
        B = 65536
        prob = P.make_batch(B, horizon=N, n_footsteps=6, seed=P.SEED)
        # every input resident in HBM before timing (the phase corners, times and references,
        # the initial DCMs, omega and the swing-foot knots)
        res = {k: torch.from_numpy(prob[k]).to(dev)
               for k in ("xi_init", "omega", "nphases", "phase_begin", "phase_end", "phase_corners",
                         "phase_ncorners", "phase_ref")}
        t = lambda k: res[k]
        d = {k: t(k) for k in ("xi_init", "omega")}
        kt, kp, tq = (torch.from_numpy(a).to(dev) for a in P.swing_splines(prob, queries=32))
        params = native.default_params(N)
        out = {}
        Pn = prob["phase_begin"].shape[1]

        def step():
            # ConvexHullHelper on every phase's support polygon (blf_hull2d_hrep), the QPs read
            # their knots' constraints and references from that phase table
            # (blf_dcm_mpc_solve_phased; --expand-path: blf_dcm_phase_expand + blf_dcm_mpc_solve),
            # then the swing-foot splines
            table = h.phase_table(t("nphases"), t("phase_begin"), t("phase_end"), t("phase_corners"),
                                  t("phase_ncorners"), ref=t("phase_ref"))
            if args.expand_path:
                w = h.dcm_phase_expand(table, 0, prob["dt"], N)
                w.update(d)
                out["qp"] = h.dcm_mpc_solve(w, params)
            else:
                out["qp"] = h.dcm_mpc_solve_phased(table, 0, d["xi_init"], d["omega"], params,
                                                   out=out.get("qp"))
            coeffs = h.quintic_fit(kt, kp)
            out["sp"] = h.quintic_eval(kt, coeffs, tq)

        sec = _timed(step, args.steps, args.warmup)
        assert int((out["qp"]["status"] != 0).sum()) == 0
        line = {"metric": "DCM-MPC pipeline solves/sec (hull H-rep + QP + swing splines)",
                "value": B / sec, "unit": "QP/s", "n_gpus": 1, "ms_per_step": sec * 1e3,
                "steps": args.steps, "warmup": args.warmup, "dtype": "f64",
                "config": {"workload": f"configs[2]: batch={B}, horizon={N}, {B * Pn} phase "
                                       f"support polygons (hull H-rep) "
                                       f"{'expanded to the knots in HBM' if args.expand_path else 'read by the QP kernel (phase-indexed)'}, "
                                       f"{kt.shape[0]} swing splines x 32 queries",
                           "batch_per_gpu": B}}
        if not args.no_cpu:
            line["cpu_baseline"] = pipeline_cpu(N)
    else:
        return closed_loop(args, h, dev)
    emit(line)


def c5_shard(model, rank, B, N, periods):
    """Rank `rank`'s robots of configs[4]: the plans of problems [rank B, (rank + 1) B) (8
    footsteps, a standing start longer than the run) and standing states of seed 1000 + rank."""
    from blf import problems as P
    from blf import robot
    plan = P.make_batch(B, horizon=N + periods, n_footsteps=8, seed=P.SEED, start=rank * B,
                        first_ds=periods + 10)
    return plan, robot.standing_states(model, B, seed=1000 + rank)


def closed_loop(args):
    """configs[4]: the closed loop of the DCM-MPC planner and the 30-DoF floating-base robot with
    two ContinuousContactModel feet (blf/closed_loop.py), B = 16384 robots
    per GPU, one process per GPU over disjoint robot shards (no data-path collective).  One step =
    one 20 ms control period of every robot: its DCM -> the plan's xi_init, the warm-started
    plan window, the plan's first VRP -> joint references, the reference schedule's ForwardEuler
    steps (1 ms each, 19 steps = 20 ms of robot time, blf/closed_loop.py fixed_step_schedule) of
    the dynamics with the joint impedance.  The loop runs from a standing start; warmup periods first,
    then the timed ones, stream-ordered and synchronised once.

    BLF_C5_ORACLE=1 (with BLF_BENCH_BACKEND=gloo) rehearses this multi-rank path on the CPU: every
    rank runs the CPU restatement of the loop (oracle/closed_loop.py, compiled) over its shard
    through the same sharding, barriers and max-over-ranks timing (tests/test_distributed.py);
    --dump-state writes each rank's final robot state."""
    import numpy as np
    import torch
    import torch.distributed as dist
    from blf import closed_loop as DL
    from blf import robot
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    backend = os.environ.get("BLF_BENCH_BACKEND", "nccl")
    on_cpu = os.environ.get("BLF_C5_ORACLE") == "1"
    if on_cpu and backend != "gloo":
        sys.exit("bench.py: BLF_C5_ORACLE=1 runs on the CPU and needs BLF_BENCH_BACKEND=gloo")
    B = args.batch if args.batch != 4096 else 16384   # configs[4]: 16 384 robots per GPU
    N, S = args.horizon, args.warmup + args.steps
    model = robot.humanoid24()
    plan, st = c5_shard(model, rank, B, N, S)
    if on_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import closed_loop as CL
        if world > 1:
            dist.init_process_group("gloo")
        sync = lambda: None
        loops = [CL.OracleLoop(model, plan, st, robot.sole_null_poses(model, st),
                               robot.posture_law_arrays(model), DL.CONTACT_PARAMS, horizon=N,
                               compiled=True, threads=max(1, cpu_threads() // max(1, world)))]
        state_of = lambda lp: lp.state
        dt_ms, T, dT = float(plan["dt"]), loops[0].T, loops[0].dT
    else:
        from blf import native
        local = int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())
        if world > 1:
            torch.cuda.set_device(local)
            if backend == "nccl":
                dist.init_process_group("nccl", device_id=torch.device("cuda", local))
            else:
                dist.init_process_group(backend)
        torch.cuda.set_device(local)
        sync = torch.cuda.synchronize
        h = native.Handle(local)
        # the robots in G groups, each closed loop on its own stream (--c5-groups, default 2): at
        # horizon 100 every robot's period is the same computation as in one group
        # (DL.split_groups states when); two groups let one group's plan tail (the interior
        # point kernel's few uncapturable windows) run beside the other group's kernels
        # 
        loops = DL.split_groups(h, model, plan, st, args.c5_groups, horizon=N)
        for lp in loops:
            lp.expand_path = args.expand_path
        state_of = lambda lp: {k: v.cpu().numpy() for k, v in lp.state.items()}
        dt_ms, T, dT = loops[0].dt, loops[0].T, loops[0].dT
    loop = loops[0]
    for _ in range(args.warmup):
        for lp in loops:
            lp.period()
    if not on_cpu:   # the dynamics kernel's launches timed on their own streams (roofline below)
        for lp in loops:
            lp.dyn_events = []
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    statuses = []
    for _ in range(args.steps):
        for lp in loops:
            out = lp.period()
            if on_cpu:
                statuses.append(torch.from_numpy(np.asarray(out["status"], dtype=np.int64)))
            else:
                with torch.cuda.stream(lp.stream or torch.cuda.current_stream()):   # after the group's solve
                    statuses.append(out["status"].clone())
    sync()
    if world > 1:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=("cuda" if backend == "nccl" else "cpu"))
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    states = [state_of(lp) for lp in loops]
    finite = all(bool(np.isfinite(v).all()) for s_ in states for v in s_.values())
    assert finite, "non-finite robot state in the closed loop"
    if args.dump_state:
        os.makedirs(args.dump_state, exist_ok=True)
        np.savez(os.path.join(args.dump_state, f"c5_state_rank{rank}.npz"),
                 **{k: np.concatenate([s_[k] for s_ in states]) for k in states[0]})
    stat = torch.bincount(torch.cat(statuses).to(torch.int64).cpu(), minlength=4)[:4].to(torch.float64)
    z = np.concatenate([s_["base_pos"][:, 2] for s_ in states])
    zr = torch.tensor([-z.min(), z.max(), 0.0 if finite else 1.0], dtype=torch.float64)
    if world > 1:   # the whole job's statuses and heights (outside the timed region)
        dev = "cuda" if backend == "nccl" else "cpu"
        stat, zr = stat.to(dev), zr.to(dev)
        dist.all_reduce(stat, op=dist.ReduceOp.SUM)
        dist.all_reduce(zr, op=dist.ReduceOp.MAX)
    stat, zr = stat.cpu().numpy().astype(np.int64), zr.cpu().numpy()
    finite = bool(finite and zr[2] == 0.0)
    steps = DL.fixed_step_schedule(0.0, T, dT)
    nsteps = len(steps)
    robot_ms = sum(steps) * 1e3
    if rank == 0:
        line = {"metric": "closed-loop control periods/sec (DCM-MPC + 30-DoF floating-base "
                          "dynamics with 2 ContinuousContactModel feet, configs[4])",
                "value": world * B * args.steps / elapsed, "unit": "robot-periods/s",
                "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
                "scaling": "weak", "dtype": "f64", "data": "synthetic (standing start, 8-footstep plans)",
                "qp_status_counts": {"solved": int(stat[0]), "max_iter": int(stat[1]),
                                     "numerical": int(stat[2]), "bad_facets": int(stat[3])},
                "state_finite": finite,
                "base_height_range": [float(-zr[0]), float(zr[1])],
                "robot_time_per_period_ms": robot_ms,
                "config": {"workload": f"configs[4]: {B} robots per GPU x {world} GPU(s), {dt_ms * 1e3:g} ms control "
                                       f"period = one knot of a horizon-{N} warm-started plan + "
                                       f"{nsteps} ForwardEuler steps of the 6+24 DoF dynamics "
                                       f"(integrate(0, {T * 1e3:g} ms) at dT = {dT * 1e3:g} ms: "
                                       f"{robot_ms:g} ms of robot time, the reference schedule)",
                           "batch_per_gpu": B, "parallelism": f"shard{world} (independent robots)",
                           "stream_groups": len(loops)}}
        if on_cpu:
            line["device"] = "CPU rehearsal (BLF_C5_ORACLE=1: oracle/closed_loop.py on every rank)"
        else:
            ev = [e for lp in loops for e in lp.dyn_events]
            kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / len(ev)
            line["roofline"] = fbd_roofline(kernel_ms, B // len(loops))
        if not args.no_cpu:
            line["cpu_baseline"] = closed_loop_cpu(args, model, N)
        emit(line)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def pipeline_cpu(N, B=65536):
    """configs[2] on the CPU: the SAME 65 536 problems as the device step (same generator, seed and
    size), the same stages, each on every CPU this process may use (the oracle's C batch drivers,
    no Python per item):
    the hull of every phase polygon, the phase expansion of every window, the QPs (sequential
    recursions, one problem per thread) and the swing splines (fit + 32 queries)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    from blf import problems as P
    prob = P.make_batch(B, horizon=N, n_footsteps=6, seed=P.SEED)
    kt, kp, tq = P.swing_splines(prob, queries=32)
    threads = cpu_threads()
    prm = O.default_params(N, sequential=1)
    Bq, Pn, C = prob["phase_corners"].shape[:3]

    def run():
        t0 = time.perf_counter()
        A, b, nf = O.hull2d_hrep_batch(prob["phase_corners"].reshape(Bq * Pn, C, 2),
                                       prob["phase_ncorners"].reshape(Bq * Pn), 8, threads=threads)
        table = dict(nphases=prob["nphases"], phase_begin=prob["phase_begin"],
                     phase_end=prob["phase_end"], phase_A=A.reshape(Bq, Pn, 8, 2),
                     phase_b=b.reshape(Bq, Pn, 8), phase_nf=nf.reshape(Bq, Pn),
                     phase_ref=prob["phase_ref"])
        w = O.dcm_phase_expand_batch(table, 0, prob["dt"], N, threads=threads)
        w.update(xi_init=prob["xi_init"], omega=prob["omega"])
        t1 = time.perf_counter()
        st, _, _, _ = O.dcm_mpc_solve_batch(w, params=prm, threads=threads)
        t2 = time.perf_counter()
        O.quintic_batch(kt, kp, tq, threads=threads)
        t3 = time.perf_counter()
        assert (st == 0).all()
        return t1 - t0, t2 - t1, t3 - t2

    run()   # warm-up
    reps = sorted((run() for _ in range(3)), key=sum)
    (ta, tb, tc) = reps[len(reps) // 2]          # the median run
    el = ta + tb + tc
    return {"value": B / el, "unit": "QP/s", "cores": threads, "kind": "port",
            "sample": f"the device step's {B} problems on {threads} threads, median of 3 runs after a warm-up: "
                      f"{Bq * Pn} phase hulls + {B} window expansions {ta:.3f} s, QPs {tb:.3f} s "
                      f"(oracle sequential mode), {kt.shape[0]} splines x 32 queries {tc:.3f} s "
                      f"(oracle C batch drivers)"}


def receding_cpu(N, tol_polish, B=4096, windows=20):
    """The receding horizon on the CPU, a bounded sample: B plans advanced `windows` windows, each
    window expanded from the phase table and solved warm from the previous one (the oracle's C
    batch drivers on every thread this process may use, sequential recursions per problem)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np
    import oracle as O
    from blf import problems as P
    prob = P.make_batch(B, horizon=N + windows + 1, n_footsteps=8, seed=P.SEED)
    threads = cpu_threads()
    prm = O.default_params(N, sequential=1, tol_polish=tol_polish)
    Bq, Pn, C = prob["phase_corners"].shape[:3]
    A, b, nf = O.hull2d_hrep_batch(prob["phase_corners"].reshape(Bq * Pn, C, 2),
                                   prob["phase_ncorners"].reshape(Bq * Pn), 8, threads=threads)
    table = dict(nphases=prob["nphases"], phase_begin=prob["phase_begin"],
                 phase_end=prob["phase_end"], phase_A=A.reshape(Bq, Pn, 8, 2),
                 phase_b=b.reshape(Bq, Pn, 8), phase_nf=nf.reshape(Bq, Pn),
                 phase_ref=prob["phase_ref"])
    xi0, prev = prob["xi_init"], None

    def window(s):
        nonlocal xi0, prev
        w = O.dcm_phase_expand_batch(table, s, prob["dt"], N, threads=threads)
        w.update(xi_init=xi0, omega=np.ascontiguousarray(prob["omega"][:, s:s + N]))
        pv, pl = (None, None) if prev is None else prev
        st, xi, vrp, _, lam = O.dcm_mpc_solve_batch_warm(w, vrp_ws=pv, lam_ws=pl, shift=1,
                                                         floor=1e-3, params=prm, threads=threads)
        prev, xi0 = (vrp, lam), np.ascontiguousarray(xi[:, 1])
        return st

    window(0)   # the cold first window, untimed (the device bench also times warm windows only)
    t0 = time.perf_counter()
    for s in range(1, windows + 1):
        st = window(s)
    el = time.perf_counter() - t0
    return {"value": B * windows / el, "unit": "QP/s", "cores": threads, "kind": "port",
            "sample": f"{B} plans x {windows} warm windows in {el:.2f} s on {threads} threads "
                      f"(phase expansion + warm solve per window, oracle C batch drivers, "
                      f"sequential mode), {int((st != 0).sum())} unsolved in the last window"}


def closed_loop_cpu(args, model, N, periods=3):
    """The CPU composition of the same loop, compiled: oracle/closed_loop.py OracleLoop with the C
    restatements of the centre of mass and of the impedance-driven floating-base dynamics
    (oracle/blf_oracle_fbd.c) and the C oracle's warm QP, all robots spread over the host's
    threads; a bounded sample of 256 robots per thread for `periods` periods."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import closed_loop as CL
    from blf import closed_loop as DL
    from blf import problems as P
    from blf import robot
    threads = cpu_threads()
    robots = 256 * threads
    plan = P.make_batch(robots, horizon=N + periods, n_footsteps=8, seed=P.SEED,
                        first_ds=periods + 10)
    st = robot.standing_states(model, robots, seed=1000)
    ref = CL.OracleLoop(model, plan, st, robot.sole_null_poses(model, st),
                        robot.posture_law_arrays(model), DL.CONTACT_PARAMS, horizon=N,
                        compiled=True, threads=threads)
    ref.period()   # warm-up (the first period is the cold solve, as on the device)
    nsteps = len(DL.fixed_step_schedule(0.0, ref.T, ref.dT))
    t0 = time.perf_counter()
    for _ in range(periods - 1):
        ref.period()
    el = time.perf_counter() - t0
    n = robots * (periods - 1)
    return {"value": n / el, "unit": "robot-periods/s", "cores": threads, "kind": "port",
            "sample": f"{robots} robots x {periods - 1} warm periods in {el:.2f} s on {threads} "
                      f"threads (oracle/closed_loop.py compiled: C centre of mass + {nsteps} impedance "
                      f"Euler steps of the C floating-base dynamics per period, the C oracle's "
                      f"warm QP; gcc -O3)"}


def single_solve_latency(args, h, dev):
    """configs[0]: one TimeVaryingDCMPlanner solve (4 footsteps, 50-knot horizon), the reference's
    Planners-test case.  Latency of one blf_dcm_mpc_solve (inputs resident, launch to completion,
    median of 50) next to the CPU restatement on one thread (oracle sequential mode), same
    problem.  A batch of one leaves 255 of 256 CUs idle: the GPU path is built for batches."""
    import numpy as np
    import torch
    from blf import native
    from blf import problems as P
    N = 50
    prob = P.make_batch(1, horizon=N, n_footsteps=4, seed=P.SEED)
    d = {k: torch.from_numpy(prob[k]).to(dev) for k in ("xi_init", "omega", "xi_ref", "vrp_ref")}
    A, b, nf = h.assemble_constraints(torch.from_numpy(prob["corners"]).to(dev),
                                      torch.from_numpy(prob["ncorners"]).to(dev))
    d.update(A=A, b=b, nfacets=nf)
    params = native.default_params(N)
    out = h.dcm_mpc_solve(d, params)
    torch.cuda.synchronize()
    lat = []
    for _ in range(args.warmup + 50):
        t0 = time.perf_counter()
        h.dcm_mpc_solve(d, params, out=out)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    py_us = float(np.median(lat[args.warmup:])) * 1e6
    # the drop-in boundary: the C-ABI call with its argument structs held (what the C++
    # TimeVaryingDCMPlanner adapter pays per solve) + hipStreamSynchronize, no Python marshalling
    import ctypes
    solve, stream = h.prepare_dcm_mpc_solve(d, params, out)
    hip = ctypes.CDLL("libamdhip64.so.7")   # the runtime torch and libblf.so already share
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    sync = hip.hipStreamSynchronize
    lat = []
    for _ in range(args.warmup + 200):
        t0 = time.perf_counter()
        solve()
        if sync(stream) != 0:
            raise RuntimeError("hipStreamSynchronize failed")
        lat.append(time.perf_counter() - t0)
    gpu_us = float(np.median(lat[args.warmup:])) * 1e6
    # the same call timed on the device (HIP events on the stream the solve is enqueued on): the
    # kernels alone, without the host's argument marshalling, launch and synchronisation.  A spin
    # kernel ahead of the start event keeps the device busy while the host enqueues the solve, so
    # the start event is reached only when the solve's kernels are already queued behind it.
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(100)]
    for i in range(50):
        torch.cuda._sleep(1 << 20)
        ev[2 * i].record()
        h.dcm_mpc_solve(d, params, out=out)
        ev[2 * i + 1].record()
        torch.cuda.synchronize()
    dev_us = float(np.median([ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(50)])) * 1e3
    assert int(out["status"][0]) == 0
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    host = dict(prob)
    for k in ("A", "b", "nfacets"):
        host[k] = d[k].cpu().numpy()
    prm = O.default_params(N, sequential=1)
    # the same problem 200 times through the C batch entry on one thread: C time per solve,
    # without per-call Python marshalling
    rep = {k: np.ascontiguousarray(np.repeat(np.asarray(host[k]), 200, axis=0))
           for k in ("xi_init", "omega", "xi_ref", "vrp_ref", "A", "b", "nfacets")}
    O.dcm_mpc_solve_batch(rep, params=prm, threads=1)
    t1 = time.perf_counter()
    st, _, _, it = O.dcm_mpc_solve_batch(rep, params=prm, threads=1)
    cpu_us = (time.perf_counter() - t1) / 200 * 1e6
    assert (st == 0).all()
    line = {"metric": "single DCM-MPC solve latency (configs[0]: 4 footsteps, horizon 50)",
            "value": gpu_us, "unit": "us", "n_gpus": 1, "higher_is_better": False,
            "dtype": "f64", "ipm_iters": int(out["iters"][0]), "polished": int(out["polished"][0]),
            "device_us": dev_us, "python_call_us": py_us,
            "cpu_baseline": {"value": cpu_us, "unit": "us", "cores": 1, "kind": "port",
                             "sample": "200 solves of the same problem in one C batch call, "
                                       "oracle/blf_oracle.c sequential mode, gcc -O3, one thread"},
            "config": {"workload": "configs[0]: batch=1, 4 footsteps, horizon=50; value = one "
                                   "blf_dcm_mpc_solve C-ABI call (argument structs held, inputs "
                                   "resident) to the end of hipStreamSynchronize, median of 200; "
                                   "python_call_us = the same through the Python wrapper; "
                                   "device_us = the kernels alone (HIP events)"}}
    emit(line)


def phase_expand_bytes(P, N, M):
    """Algorithmic bytes of blf_dcm_phase_expand per problem: the phase table read once
    (nphases, begin/end, A rows, b, counts, reference points) and the window written."""
    return 4 + P * (16 + 24 * M + 4 + 16) + N * (24 * M + 4 + 16) + 16 * (N + 1)


def three_contact(args, h, dev):
    """Plans with three-contact phases: the reference ContactPhaseList test's
    three lists (src/Planners/tests/ContactPhaseListTest.cpp:32-47) with the feet turned out and
    a hand support ahead, B = 4096 plans, N = 50 knots of 0.1 s, max_facets 16 (hulls of up to 9
    facets).  Two lines' worth in one: the cold phase-indexed solve of window 0, repeated on the
    same inputs (cold QP/s), and the receding horizon, every window warm-started from the last
    (blf_dcm_mpc_solve_phased; --expand-path: blf_dcm_phase_expand + blf_dcm_mpc_solve_warm, with
    BLF_QP_SINGLE_KERNEL=1 the interior point kernel alone)."""
    import torch
    from blf import native
    from blf import problems as P
    B, N, M = args.batch, 50, 16
    S = args.warmup + 2 * args.steps + 1
    knots = max(75, N + S)
    prob = P.three_contact_plan(B, knots=knots, seed=P.SEED)
    t = lambda k: torch.from_numpy(prob[k]).to(dev)
    table = h.phase_table(t("nphases"), t("phase_begin"), t("phase_end"), t("phase_corners"),
                          t("phase_ncorners"), max_facets=M, ref=t("phase_ref"))
    omega_full = t("omega")
    params = native.default_params(N, max_facets=M, dt=prob["dt"])
    params.tol_polish = args.tol_polish if args.tol_polish is not None else 1e-4
    xi0 = t("xi_init")
    e64 = lambda *shape: torch.empty(shape, dtype=torch.float64, device=dev)
    e32 = lambda *shape: torch.empty(shape, dtype=torch.int32, device=dev)
    window = dict(omega=e64(B, N), xi_ref=e64(B, N + 1, 2), vrp_ref=e64(B, N, 2), A=e64(B, N, M, 2),
                  b=e64(B, N, M), nfacets=e32(B, N))
    newbuf = lambda: dict(xi=e64(B, N + 1, 2), vrp=e64(B, N, 2), status=e32(B), iters=e32(B),
                          polished=e32(B), passes=e32(B), lam=e64(B, N, M), window=window)

    def solve(s, xi, warm, out):
        if args.expand_path:
            w = h.dcm_phase_expand(table, s, prob["dt"], N)
            w.update(xi_init=xi, omega=omega_full[:, s:s + N].contiguous())
            return h.dcm_mpc_solve(w, params, out=out, warm=warm, lambda_out=True)
        return h.dcm_mpc_solve_phased(table, s, xi, omega_full[:, s:s + N], params, warm=warm, out=out,
                                      lambda_out=True)

    # cold: window 0 from the plans' initial DCMs, the same inputs every step
    cold = newbuf()
    for _ in range(args.warmup):
        solve(0, xi0, None, cold)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        solve(0, xi0, None, cold)
    torch.cuda.synchronize()
    sec_cold = (time.perf_counter() - t0) / args.steps
    cold_unsolved = int((cold["status"] != 0).sum())
    cold_passes = float(cold["passes"].float().mean())
    cold_ipm = int((cold["iters"] > 0).sum())
    # warm: the receding horizon, window s + 1 warm-started from window s
    bufs = [newbuf() for _ in range(S)]
    state = dict(xi=xi0.clone(), prev=None, s=0)

    def step():
        s = state["s"]
        warm = None
        if state["prev"] is not None:
            warm = dict(vrp=state["prev"]["vrp"], lam=state["prev"]["lam"], shift=1, floor=1e-3)
        out = solve(s, state["xi"], warm, bufs[s])
        state["xi"] = out["xi"][:, 1].contiguous()
        state["prev"] = out
        state["s"] = s + 1

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    sec_warm = (time.perf_counter() - t0) / args.steps
    statuses = torch.stack([bufs[i]["status"] for i in range(state["s"])])
    warm_unsolved = int((statuses != 0).sum())
    warm_passes = float(torch.stack([bufs[i]["passes"] for i in range(1, state["s"])]).float().mean())
    nf = table["phase_nf"]
    line = {"metric": "three-contact DCM-MPC QP solves/sec (cold window; warm receding horizon)",
            "value": B / sec_cold, "unit": "QP/s", "n_gpus": 1, "ms_per_step": sec_cold * 1e3,
            "warm_value": B / sec_warm, "warm_ms_per_step": sec_warm * 1e3,
            "steps": args.steps, "warmup": args.warmup, "dtype": "f64",
            "cold": {"unsolved": cold_unsolved, "mean_active_set_passes": cold_passes,
                     "qps_to_interior_point": cold_ipm},
            "warm": {"windows": state["s"], "unsolved": warm_unsolved,
                     "mean_active_set_passes": warm_passes},
            "max_hull_facets": int(nf.max()),
            "path": ("blf_dcm_phase_expand + blf_dcm_mpc_solve_warm" if args.expand_path else
                     "blf_dcm_mpc_solve_phased") +
                    (" (interior point kernel alone, BLF_QP_SINGLE_KERNEL=1)"
                     if os.environ.get("BLF_QP_SINGLE_KERNEL") == "1" else ""),
            "data": "synthetic (the reference ContactPhaseList test's three lists, randomised poses)",
            "config": {"workload": "three-contact plans, B=4096, horizon=50, dt=0.1, max_facets=16",
                       "batch": B, "horizon": N, "max_facets": M}}
    emit(line)


def receding_horizon(args, h, dev):
    """TimeVaryingDCMPlanner::advance() on the device, B = 4096 plans: per step the knot -> phase
    expansion of the window (blf_dcm_phase_expand), the warm-started solve
    (blf_dcm_mpc_solve_warm, shifted previous VRPs and multipliers), and xi_1 -> next xi_init.
    The phase polygons are built once (blf_hull2d_hrep over the phases) before timing."""
    import torch
    from blf import native
    from blf import problems as P
    B, N = args.batch, args.horizon
    S = args.warmup + 2 * args.steps + 1   # warmup, timed steps, then the steps that take statistics
    prob = P.make_batch(B, horizon=N + S, n_footsteps=8, seed=P.SEED)
    t = lambda k, dt=None: torch.from_numpy(prob[k]).to(dev)
    table = h.phase_table(t("nphases"), t("phase_begin"), t("phase_end"), t("phase_corners"),
                          t("phase_ncorners"), ref=t("phase_ref"))
    omega_full = t("omega")
    M = table["phase_b"].shape[2]
    params = native.default_params(N, max_facets=M)
    # TimeVaryingDCMPlanner's trigger for warm-started windows (1e-4; the cold default is 3e-4)
    params.tol_polish = args.tol_polish if args.tol_polish is not None else 1e-4
    stream = torch.cuda.current_stream()
    state = dict(xi0=t("xi_init").clone(), prev=None, s=0)
    # one output buffer per window (S x ~39 MB at B = 4096, allocated here, before any timing), so
    # that every window's statuses and iteration counts survive to the checks after the clock
    # stops with no copy in the timed loop; the window scratch (read only by the IPM stage of the
    # same call) is shared
    e64 = lambda *shape: torch.empty(shape, dtype=torch.float64, device=dev)
    e32 = lambda *shape: torch.empty(shape, dtype=torch.int32, device=dev)
    window = dict(omega=e64(B, N), xi_ref=e64(B, N + 1, 2), vrp_ref=e64(B, N, 2), A=e64(B, N, M, 2),
                  b=e64(B, N, M), nfacets=e32(B, N))
    bufs = [dict(xi=e64(B, N + 1, 2), vrp=e64(B, N, 2), status=e32(B), iters=e32(B),
                 polished=e32(B), lam=e64(B, N, M), window=window) for _ in range(S)]
    iters = []
    evs = []

    def step(timed=False):
        s = state["s"]
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if timed else None
        if timed:
            evs.append(ev)
            ev[0].record(stream)
        cur = s
        warm = None
        if state["prev"] is not None:
            warm = dict(vrp=state["prev"]["vrp"], lam=state["prev"]["lam"], shift=1, floor=1e-3)
        if args.expand_path:
            w = h.dcm_phase_expand(table, s, prob["dt"], N)
            if timed:
                ev[1].record(stream)
            w.update(xi_init=state["xi0"], omega=omega_full[:, s:s + N].contiguous())
            if timed:
                ev[2].record(stream)
            out = h.dcm_mpc_solve(w, params, out=bufs[cur], warm=warm, lambda_out=True)
        else:   # one call: the window read from the phase table, omega as a strided view
            if timed:
                ev[1].record(stream)
                ev[2].record(stream)
            out = h.dcm_mpc_solve_phased(table, s, state["xi0"], omega_full[:, s:s + N], params,
                                         warm=warm, out=bufs[cur], lambda_out=True)
        if timed:
            ev[3].record(stream)
        bufs[cur] = out
        state["xi0"] = out["xi"][:, 1].contiguous()
        state["prev"] = out
        state["s"] = s + 1
        if timed:
            iters.append(out["iters"])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # advance() is stream-ordered (no host round trip), so the steps are enqueued back to back and
    # the host synchronizes once, after the last one.  The timed steps are advance() alone; the
    # per-step events and iteration copies (bookkeeping, host work per step) run on the next
    # args.steps windows, after the clock has stopped.
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    sec = (time.perf_counter() - t0) / args.steps
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    expand_ms = [e[0].elapsed_time(e[1]) for e in evs]
    solve_ms = [e[2].elapsed_time(e[3]) for e in evs]
    # every window of the run (warmup, timed, bookkeeping): solved
    statuses = torch.stack([bufs[i]["status"] for i in range(state["s"])])
    unsolved = int((statuses != 0).sum())
    assert unsolved == 0, f"{unsolved} unsolved QPs over {state['s']} windows"
    it = torch.stack(iters).float()
    Pn = table["phase_begin"].shape[1]
    line = {"metric": "receding-horizon DCM-MPC advance()/sec (phase expansion + warm-started QP)",
            "value": B / sec, "unit": "QP/s", "n_gpus": 1, "ms_per_step": sec * 1e3,
            "steps": args.steps, "warmup": args.warmup, "dtype": "f64",
            "mean_ipm_iters_warm": float(it.mean()),
            "windows_checked": {"windows": state["s"], "qps": state["s"] * B, "unsolved": unsolved},
            # events around the solve call in the untimed bookkeeping pass: the GPU waits there
            # for the host's next launch, so this is an upper bound on the solve's kernel time
            "solve_event_ms_median": sorted(solve_ms)[len(solve_ms) // 2],
            "path": "blf_dcm_phase_expand + blf_dcm_mpc_solve_warm" if args.expand_path else
                    "blf_dcm_mpc_solve_phased (window read from the phase table in the QP kernel)",
            "config": {"workload": f"batch={B} plans (8 footsteps, {Pn} phases), horizon={N}, "
                                   f"window moved one knot per step, warm start shift 1 floor 1e-3",
                       "batch_per_gpu": B}}
    if not args.no_cpu:
        line["cpu_baseline"] = receding_cpu(N, params.tol_polish)
    if args.expand_path:
        ex_ms = sorted(expand_ms)[len(expand_ms) // 2]
        ex_gbs = phase_expand_bytes(Pn, N, M) * B / (ex_ms * 1e-3) / 1e9
        line["phase_expand"] = {"kernel_ms_median": ex_ms, "bytes_per_problem":
                                phase_expand_bytes(Pn, N, M), "achieved_gbs": ex_gbs,
                                "frac_hbm": ex_gbs / HBM_PEAK_GBS}
    emit(line)


if __name__ == "__main__":
    main()
