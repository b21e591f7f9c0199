"""Multi-GPU sharding of independent DCM-MPC problems.

One process per GPU.  Problems are independent, so each rank owns a contiguous shard of the
global batch and solves it with no data-path collective; the only exchange is the gather of the
solutions to rank 0 (RCCL over xGMI on MI355X — torch.distributed backend "nccl" is RCCL on ROCm;
"gloo" in the CPU tests).  The payload per problem is xi (2(N+1)), vrp (2N), status and
iteration count packed into one fp64 row, so one collective moves everything.
"""
import torch
import torch.distributed as dist


def shard(per_rank, rank):
    """Weak scaling: rank r owns global problems [r * per_rank, (r + 1) * per_rank)."""
    return rank * per_rank, per_rank


def pack(out):
    B = out["xi"].shape[0]
    return torch.cat([out["xi"].reshape(B, -1), out["vrp"].reshape(B, -1),
                      out["status"].to(torch.float64)[:, None],
                      out["iters"].to(torch.float64)[:, None]], dim=1).contiguous()


def unpack(payload, horizon):
    N = horizon
    B = payload.shape[0]
    xi = payload[:, :2 * (N + 1)].reshape(B, N + 1, 2)
    vrp = payload[:, 2 * (N + 1):2 * (N + 1) + 2 * N].reshape(B, N, 2)
    status = payload[:, -2].to(torch.int32)
    iters = payload[:, -1].to(torch.int32)
    return dict(xi=xi, vrp=vrp, status=status, iters=iters)


def gather_solutions(out, horizon, dst=0):
    """Gather every rank's solution dict to `dst` (equal shard sizes).  Returns the concatenated
    solution on dst, None elsewhere."""
    payload = pack(out)
    world = dist.get_world_size()
    bufs = [torch.empty_like(payload) for _ in range(world)] if dist.get_rank() == dst else None
    dist.gather(payload, bufs, dst=dst)
    if dist.get_rank() != dst:
        return None
    return unpack(torch.cat(bufs, dim=0), horizon)
