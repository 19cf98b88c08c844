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


def exchange_sizes(n: int, group=None) -> list[int]:
    """Every rank's row count (one small all_gather; call once per layout, not per step)."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([int(n)], dtype=torch.int64, device=dev)
    parts = [torch.zeros_like(t) for _ in range(dist.get_world_size(group))]
    dist.all_gather(parts, t, group=group)
    return [int(p.item()) for p in parts]


def gather_rows(x, group=None, sizes=None, out=None):
    """Concatenate every rank's [n_r, ...] tensor along dim 0 in rank order (all ranks get it).

    sizes: every rank's n_r (exchange_sizes, cached by the caller); without it one size exchange
    runs first.  Equal shards gather straight into `out` (allocated if None): one RCCL
    all_gather_into_tensor on GPUs, an all_gather into views of `out` on gloo; no host sync.
    Ragged shards pad to the largest shard."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    if sizes is None:
        sizes = exchange_sizes(x.shape[0], group)
    if len(sizes) != world or sizes[dist.get_rank(group)] != x.shape[0]:
        raise ValueError("sizes do not match this rank's tensor / the group")
    m = max(sizes)
    x = x.contiguous()
    if x.is_cuda and dist.get_backend(group) != "nccl":
        # gloo moves host memory: stage through the host (multi-rank rehearsal on shared GPUs)
        res = gather_rows(x.cpu(), group, sizes=sizes)
        if out is not None and out.shape == res.shape:
            return out.copy_(res)
        return res.to(x.device)
    if all(s == m for s in sizes):
        if out is None:
            out = torch.empty((world * m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        if dist.get_backend(group) == "nccl":
            dist.all_gather_into_tensor(out, x, group=group)
        else:
            dist.all_gather(list(out.chunk(world)), x, group=group)
        return out
    pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[: x.shape[0]] = x
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)], dim=0)
