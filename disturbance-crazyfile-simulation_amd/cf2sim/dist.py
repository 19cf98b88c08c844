"""Multi-GPU layout: one process per GPU, envs sharded in contiguous global-id ranges.

Envs are independent, so the physics needs no collective: rank r owns
global env ids [offset, offset + count) and every random draw is keyed by the global env id
(Philox counter = (block, rng counter, global id, tag)), which makes each env's trajectory
independent of the number of ranks.  The only exchange is optional: gathering the per-rank
observation slabs for a policy that lives elsewhere (RCCL all-gather over xGMI on GPUs, gloo on
CPU).  The reference's MPI gradient all-reduce (utils/mpi_tools.py) belongs to its learner and
stays out of scope.
"""
from __future__ import annotations


def shard_range(num_envs_total: int, rank: int, world: int) -> tuple[int, int]:
    """(env_id_offset, count) of rank's contiguous shard; the first num_envs_total % world ranks
    hold one env more."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError("bad rank/world")
    base, extra = divmod(int(num_envs_total), int(world))
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def gather_rows(x, group=None):
    """Concatenate every rank's [n_r, ...] tensor along dim 0 in rank order (all ranks get it).
    Equal shard sizes use all_gather_into_tensor (one RCCL call on GPUs); ragged shards fall back
    to a size exchange + padded all_gather."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    m = max(sizes)
    if all(s == m for s in sizes) and dist.get_backend(group) == "nccl":
        out = torch.empty((world * m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(out, x.contiguous(), group=group)
        return out
    pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]] = x
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)], dim=0)
