"""Multi-GPU layout: one process per GPU, envs sharded in contiguous global-id ranges.

Envs are independent, so the physics needs no collective: rank r owns
global env ids [offset, offset + count) and every random draw is keyed by the global env id
(Philox counter = (block, rng counter, global id, tag)), which makes each env's trajectory
independent of the number of ranks.  The only exchange is optional: gathering the per-rank
observation slabs for a policy that lives elsewhere (RCCL all-gather over xGMI on GPUs, gloo on
CPU).  The reference's MPI gradient all-reduce (utils/mpi_tools.py) belongs to its learner and
stays out of scope.

``launch_plan`` / ``run_ranks`` start one process per GPU when no launcher (torchrun) did, and
``PipelinedObsGather`` overlaps the per-step observation all-gather with the next env-step.
"""
from __future__ import annotations

import os


def launch_plan(world: int, port: int, script: str, argv: list[str], base_env: dict | None = None,
                python: str | None = None) -> list[tuple[list[str], dict]]:
    """(command, environment) of each rank when a script launches its own ranks: one fresh process
    per GPU, rank r on local GPU r, rendezvous on 127.0.0.1:port.  This is the role of the
    reference's ``mpi_fork`` (utils/mpi_tools.py:47-99, which re-runs the script under
    ``mpirun -np N``); here the ranks are started as children, never by re-executing the calling
    process, and before the caller makes any GPU call (a process that has touched the GPU must not
    exec another program)."""
    import sys
    if world < 1:
        raise ValueError("world must be >= 1")
    env0 = dict(os.environ if base_env is None else base_env)
    cmd = [python or sys.executable, "-u", script, *argv]
    plan = []
    for r in range(world):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(world), LOCAL_WORLD_SIZE=str(world),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        plan.append((list(cmd), env))
    return plan


def run_ranks(plan, timeout: float | None = None) -> int:
    """Start every rank of a launch_plan, wait for all of them and return the first non-zero exit
    code (0 if all succeeded).  If one rank fails, the others are terminated (their own process
    groups only) so a collective never waits for a dead peer."""
    import signal
    import subprocess
    import time
    procs = [subprocess.Popen(cmd, env=env, start_new_session=True) for cmd, env in plan]
    rc, t0 = 0, time.monotonic()
    try:
        while procs:
            for p in list(procs):
                code = p.poll()
                if code is None:
                    continue
                procs.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in procs:
                        os.killpg(q.pid, signal.SIGTERM)
            if timeout is not None and time.monotonic() - t0 > timeout:
                for q in procs:
                    os.killpg(q.pid, signal.SIGKILL)
                return rc or 124
            time.sleep(0.05)
    finally:
        for q in procs:
            if q.poll() is None:
                os.killpg(q.pid, signal.SIGKILL)
    return rc


class PipelinedObsGather:
    """Per-step all-gather of the observation slab ("RCCL all-gather over
    xGMI only for the returned observation tensor"), overlapped with the next env-step.

    ``depth`` observation buffers rotate: env-step k writes ``buffer()`` on the compute stream and
    ``publish()`` starts the all-gather of that buffer on a side stream, so the gather of step k
    runs while step k+1 computes.  Before step k+depth overwrites a buffer, the compute stream (not
    the host) waits for the gather that read it.  ``publish()`` returns the [world * n, D] tensor
    the gather fills; it is complete once ``wait(k)`` or ``drain()`` returned and stays valid until
    the gather of step k + depth reuses it.  On gloo (CPU rehearsal of the multi-rank path) the
    gather stages through the host and completes inside ``publish()``."""

    def __init__(self, n: int, obs_dim: int, device, group=None, depth: int = 2):
        import torch
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.nccl = dist.get_backend(group) == "nccl"
        self.depth = int(depth)
        self.obs = [torch.empty(n, obs_dim, device=device) for _ in range(self.depth)]
        self.out = [torch.empty(self.world * n, obs_dim, device=device) for _ in range(self.depth)]
        self.sizes = [n] * self.world
        self.comm = torch.cuda.Stream(device=device) if self.nccl else None
        self.work = [None] * self.depth
        self.k = 0

    def buffer(self):
        """The obs buffer env-step k writes; the current stream first waits (on the device) for
        the gather of step k - depth, which read it."""
        j = self.k % self.depth
        w = self.work[j]
        if w is not None:
            w.wait()
            self.work[j] = None
        return self.obs[j]

    def publish(self):
        """Start the all-gather of the buffer the current env-step wrote; returns its output."""
        import torch
        import torch.distributed as dist
        j = self.k % self.depth
        if self.nccl:
            self.comm.wait_stream(torch.cuda.current_stream(self.obs[j].device))
            with torch.cuda.stream(self.comm):
                self.work[j] = dist.all_gather_into_tensor(self.out[j], self.obs[j], group=self.group, async_op=True)
        else:
            gather_rows(self.obs[j], self.group, sizes=self.sizes, out=self.out[j])
        self.k += 1
        return self.out[j]

    def drain(self):
        """Make the current stream wait for every gather in flight."""
        for j, w in enumerate(self.work):
            if w is not None:
                w.wait()
                self.work[j] = None


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
