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
import weakref as _weakref


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


# ---- delta observation exchange (csrc/cf2sim_exchange.hip has the protocol; cf2_obs_pack /
# cf2_obs_consume / cf2_obs_rows run it on GPU tensors, the torch-op versions below on CPU tensors
# for the gloo rehearsal of the multi-rank path; both produce the same rows bit for bit) ----

PACK_BLOCK = 64       # envs per pack block: one block-table word each (the side slot of the block's first reset)
PACK_DROPPED = -1     # block-table word (int32 view of 0xFFFFFFFF): the block's resets past its quota got no slot
PACK_SCRATCH_WORDS = 32    # the spill counter of a pack (csrc/cf2sim_pack.h), past the largest packed buffer
ZERO_AHEAD = 16       # a consume zeroes the look-ahead rows of up to 16 steps after its own (CONSUME_MAX of
                      # csrc/cf2sim_exchange.hip: the native consume's count; the torch ops zero one)
NPRED_MIN = 2 * ZERO_AHEAD + 1    # cf2_xchg_register's smallest count ring when the time-out watch is on
NO_WATCH = 0xFFFFFFFF
PRED_BATCH = 4        # eager exchange: the time-out count ring is copied to the host every 4 env-steps
RUN_UNIT = 16         # native exchange: env-steps per batch of PipelinedObsGather.run (one all-gather each)


def _side(n: int, ol: int) -> int:
    """Word offset of the side entries: header, o_k rows, bitmap, block table."""
    return 4 + n * ol + (n + 31) // 32 + (n + PACK_BLOCK - 1) // PACK_BLOCK


def packed_words(n: int, ol: int, cap: int) -> int:
    """32-bit words of one rank's packed buffer (cf2_obs_packed_words)."""
    return (_side(n, ol) + cap * (ol + 5) + 3) & ~3


def default_cap(n: int) -> int:
    """Side-slab capacity: 7.5 % of the shard.  The bench workload ends 4.1 % of its episodes per
    env-step in steady state and 5.7 % at the synchronised-start peak (profiles/r02_reset_rate.json);
    a step that exceeds it NaNs the o_0 / action parts of the reset rows of the 64-env blocks that
    found no room and counts those blocks as overflows."""
    return min(int(n), max(64, (3 * n + 39) // 40))


def delta_supported(cfg) -> bool:
    """The delta rows rely on the action buffer holding only the step's action after an env-step
    (aggregate_phy_steps a multiple of buf_size, latency on: the reference's default) and on
    auto-reset (a finished env's next row is its reset row)."""
    return bool(cfg.auto_reset) and bool(cfg.use_latency) and int(cfg.aggregate_phy_steps) % int(cfg.buf_size) == 0


def _bits_to_mask(words, n):
    import numpy as np
    import torch
    b = words.contiguous().cpu().numpy().view(np.uint8)
    return torch.from_numpy(np.unpackbits(b, bitorder="little")[:n].astype(bool))


def _need(ok: bool, what: str):
    if not ok:
        raise ValueError(f"delta exchange: {what}")


def pack_obs(obs, reset, cap: int, out=None, scratch=None, next_scratch=None):
    """One rank's packed buffer (int32 [packed_words]) from its step's obs rows [n, OD] and
    auto-reset flags [n] (uint8 or bool).  GPU: scratch = this pack's side-slot counters
    (PACK_SCRATCH_WORDS int32, zeroed; a fresh zeroed one if None), next_scratch = the counters the
    next pack uses (zeroed by this one; or None).  CPU: slots are handed out in block order."""
    import numpy as np
    import torch
    n, od = obs.shape
    ol = od // 2 - 4
    words = packed_words(n, ol, cap)
    if out is None:
        out = torch.zeros(words, dtype=torch.int32, device=obs.device)
    if obs.is_cuda:
        from . import _native
        lib = _native.load()
        if scratch is None:
            scratch = torch.zeros(PACK_SCRATCH_WORDS, dtype=torch.int32, device=obs.device)
        # the kernel indexes by these sizes: check them on the host before the launch
        _need(obs.is_contiguous() and obs.dtype == torch.float32, "obs must be contiguous float32 [n, OD]")
        _need(reset.numel() >= n and reset.is_cuda, "reset needs n flags on the GPU")
        _need(out.dtype == torch.int32 and out.is_contiguous() and out.numel() >= words and out.is_cuda,
              f"out needs {words} int32 words on the GPU")
        for name, t in (("scratch", scratch), ("next_scratch", next_scratch)):
            _need(t is None or (t.is_cuda and t.dtype == torch.int32 and t.is_contiguous()
                                and t.numel() >= PACK_SCRATCH_WORDS), f"{name} needs {PACK_SCRATCH_WORDS} int32")
        _need(next_scratch is None or next_scratch.data_ptr() != scratch.data_ptr(), "next_scratch must not be scratch")
        r8 = reset if reset.dtype == torch.uint8 else reset.to(torch.uint8)
        _native.check(lib.cf2_obs_pack(obs.data_ptr(), r8.contiguous().data_ptr(), n, ol, cap, out.data_ptr(),
                                       scratch.data_ptr(), _native.ptr(next_scratch),
                                       torch.cuda.current_stream(obs.device).cuda_stream), "cf2_obs_pack")
        return out
    r = reset.bool().cpu()
    out.zero_()
    f = out.view(torch.float32)
    f[4:4 + n * ol] = obs[:, ol + 4:2 * ol + 4].reshape(-1)
    nb = (n + 31) // 32
    bits = np.zeros(4 * nb, np.uint8)
    pb = np.packbits(r.numpy(), bitorder="little")
    bits[:pb.size] = pb
    out[4 + n * ol:4 + n * ol + nb] = torch.from_numpy(bits.view(np.int32))
    out[1], out[2], out[3] = n, ol, cap
    # side slots (csrc/cf2sim_pack.h): each 64-env block owns `quota` slots for its first resets; the
    # excess takes consecutive slots of the spill area (blocks in order here; the GPU's atomic hands
    # them out in arrival order, so only the slots differ, not the rows), or is dropped
    nblk = (n + PACK_BLOCK - 1) // PACK_BLOCK
    q = pack_quota(n, cap)
    spill_base = nblk * q
    cnt = torch.zeros(nblk, dtype=torch.int64)
    idx = torch.nonzero(r).flatten()
    cnt.index_add_(0, idx // PACK_BLOCK, torch.ones_like(idx))
    btab = torch.zeros(nblk, dtype=torch.int64)
    side, used = _side(n, ol), 0
    for b in torch.nonzero(cnt).flatten().tolist():
        c = int(cnt[b])
        first = 0
        if c > q:
            if used + c - q > cap - spill_base:
                first = PACK_DROPPED
            else:
                first = spill_base + used
                used += c - q
        btab[b] = first
        for s_, i in enumerate(idx[(idx // PACK_BLOCK) == b].tolist()):
            if s_ < q:
                slot = b * q + s_
            elif first == PACK_DROPPED:
                continue
            else:
                slot = first + s_ - q
            e = side + slot * (ol + 5)
            out[e] = i
            f[e + 1:e + 1 + ol + 4] = obs[i, :ol + 4]
    out[4 + n * ol + nb:4 + n * ol + nb + nblk] = btab.to(torch.int32)
    return out


def pack_quota(n: int, cap: int) -> int:
    """Side slots each 64-env pack block owns (PackLayout::quota): min(cap, default_cap(n)) // blocks,
    at most 64.  Capacity above the default crash budget (predicted time-outs) is all spill area."""
    return min(min(int(cap), default_cap(n)) // ((int(n) + PACK_BLOCK - 1) // PACK_BLOCK), PACK_BLOCK)


def _slots(pk, n: int, ol: int, cap: int, rs):
    """Side slot of every env (valid where rs; PACK_DROPPED where it got none) from its rank among its
    block's resets, the block's quota and the block table (cf2sim_pack.h pack_slot)."""
    import torch
    nb = (n + 31) // 32
    nblk = (n + PACK_BLOCK - 1) // PACK_BLOCK
    btab = pk[4 + n * ol + nb:4 + n * ol + nb + nblk].to(torch.int64)
    blk = torch.arange(n) // PACK_BLOCK
    c = torch.cumsum(rs.to(torch.int64), 0)
    start = torch.zeros(nblk, dtype=torch.int64)
    start[1:] = c[torch.arange(1, nblk) * PACK_BLOCK - 1]
    within = c - rs.to(torch.int64) - start[blk]
    first = btab[blk]
    q = pack_quota(n, cap)
    spill = torch.where(first == PACK_DROPPED, torch.full_like(first, PACK_DROPPED), first + within - q)
    return torch.where(within < q, blk * q + within, spill)


def consume_obs(recv, world: int, n: int, ol: int, cap: int, age, overflow=None, watch_age: int = NO_WATCH,
                pred=None, pred_next=None):
    """A receiver's per-step work (cf2_obs_consume): advance every env's age (steps since its reset;
    int16 storage of a uint16 on GPUs, int32 on the CPU, [world n]) from the gathered packed buffers
    (int32 [world * packed_words(n, ol, cap)]); count per rank into pred ([world]) the envs whose new age is watch_age (they time out L
    steps later unless they crash first); zero pred_next; count the 64-env blocks whose resets got
    no side slot into overflow."""
    import torch
    if recv.is_cuda:
        from . import _native
        lib = _native.load()
        N = world * n
        _need(recv.dtype == torch.int32 and recv.is_contiguous() and recv.numel() >= world * packed_words(n, ol, cap),
              "recv needs world * packed_words int32 words")
        _need(age.dtype == torch.int16 and age.is_contiguous() and age.numel() >= N and age.is_cuda,
              "age must be int16 (uint16 storage) [world * n] on the GPU")
        for name, t, k in (("overflow", overflow, 1), ("pred", pred, world), ("pred_next", pred_next, world)):
            _need(t is None or (t.is_cuda and t.dtype == torch.int32 and t.numel() >= k), f"{name} needs {k} int32")
        _need((pred is None) == (pred_next is None), "pred and pred_next go together")
        _native.check(lib.cf2_obs_consume(recv.data_ptr(), world, n, ol, cap, age.data_ptr(), _native.ptr(overflow),
                                          int(watch_age) & 0xFFFFFFFF, _native.ptr(pred), _native.ptr(pred_next),
                                          torch.cuda.current_stream(recv.device).cuda_stream), "cf2_obs_consume")
        return age
    words = packed_words(n, ol, cap)
    rv = recv[:world * words].reshape(world, words)
    if pred_next is not None:
        pred_next.zero_()
    for r in range(world):
        pk = rv[r]
        rs = _bits_to_mask(pk[4 + n * ol:4 + n * ol + (n + 31) // 32], n)
        sl = slice(r * n, (r + 1) * n)
        a = torch.clamp(age[sl].to(torch.int64) + 1, max=0xFFFF)
        new = torch.where(rs, torch.zeros_like(a), a)
        age[sl] = new.to(age.dtype)
        if pred is not None:
            pred[r] += int((new == watch_age).sum())
        if overflow is not None:
            nb = (n + 31) // 32
            btab = pk[4 + n * ol + nb:4 + n * ol + nb + (n + PACK_BLOCK - 1) // PACK_BLOCK]
            overflow += int((btab == PACK_DROPPED).sum())
    return age


def obs_rows(recv, cap: int, recv_prev, cap_prev: int, world: int, n: int, ol: int, age, act, act_prev, act_prev2,
             out=None, row0: int = 0, nrows: int | None = None, stride: int | None = None,
             stride_prev: int | None = None):
    """Rows [row0, row0 + nrows) of step k's global observation slab ([nrows, 2 ol + 8]) from the
    gathered packed buffers of step k (recv, capacity cap) and k - 1 (recv_prev, cap_prev), the ages
    after step k's consume_obs and the actions of steps k, k - 1, k - 2 ([world n, 4]; the history
    rules of csrc/cf2sim_exchange.hip).  The reset rows of a pack block that got no side slot have NaN
    in their o_0 / action parts.  Rank r's packed buffer starts r * stride words into recv (default:
    packed_words(n, ol, cap), one step's all-gather), likewise for recv_prev."""
    import torch
    N, od = world * n, 2 * (ol + 4)
    nrows = N - row0 if nrows is None else int(nrows)
    _need(0 <= row0 and row0 + nrows <= N, "rows out of range")
    if out is None:
        out = torch.empty(nrows, od, dtype=torch.float32, device=recv.device)
    words, wp = packed_words(n, ol, cap), packed_words(n, ol, cap_prev)
    stride = words if stride is None else int(stride)
    stride_prev = wp if stride_prev is None else int(stride_prev)
    _need(stride >= words and stride_prev >= wp, "rank strides below the packed buffer size")
    if recv.is_cuda:
        from . import _native
        lib = _native.load()
        _need(recv.dtype == torch.int32 and recv.is_contiguous() and recv.numel() >= (world - 1) * stride + words,
              "recv needs (world - 1) * stride + packed_words(cap) int32 words")
        _need(recv_prev.dtype == torch.int32 and recv_prev.is_contiguous() and recv_prev.is_cuda and
              recv_prev.numel() >= (world - 1) * stride_prev + wp, "recv_prev too short")
        _need(age.dtype == torch.int16 and age.is_contiguous() and age.numel() >= N and age.is_cuda,
              "age must be int16 (uint16 storage) [world * n] on the GPU")
        for name, t in (("act", act), ("act_prev", act_prev), ("act_prev2", act_prev2)):
            _need(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() >= N * 4,
                  f"{name} must be contiguous float32 [world * n, 4] on the GPU")
        _need(out.is_cuda and out.dtype == torch.float32 and out.is_contiguous() and out.numel() >= nrows * od,
              f"out must be contiguous float32 [{nrows}, {od}] on the GPU")
        _native.check(lib.cf2_obs_rows(recv.data_ptr(), cap, stride, recv_prev.data_ptr(), cap_prev, stride_prev, world,
                                       n, ol, age.data_ptr(), act.data_ptr(), act_prev.data_ptr(), act_prev2.data_ptr(),
                                       row0, nrows, out.data_ptr(), torch.cuda.current_stream(recv.device).cuda_stream),
                      "cf2_obs_rows")
        return out
    rv = [recv[r * stride:r * stride + words] for r in range(world)]
    pv = [recv_prev[r * stride_prev:r * stride_prev + wp] for r in range(world)]
    nan = float("nan")
    full = torch.empty(N, od)
    for r in range(row0 // n, (row0 + nrows + n - 1) // n):
        pk, f = rv[r], rv[r].view(torch.float32)
        rs = _bits_to_mask(pk[4 + n * ol:4 + n * ol + (n + 31) // 32], n)
        sl = slice(r * n, (r + 1) * n)
        o = full[sl]
        a = age[sl].to(torch.int64) & 0xFFFF
        o[:, :ol] = pv[r].view(torch.float32)[4:4 + n * ol].view(n, ol)
        o[:, ol:ol + 4] = torch.where((a >= 3)[:, None], act_prev2[sl], act[sl])
        o[:, ol + 4:2 * ol + 4] = f[4:4 + n * ol].view(n, ol)
        o[:, 2 * ol + 4:] = torch.where((a == 1)[:, None], act[sl], act_prev[sl])
        sl_ = _slots(pk, n, ol, cap, rs)
        drop = rs & (sl_ == PACK_DROPPED)
        o[drop, :ol + 4] = nan
        o[drop, 2 * ol + 4:] = nan
        side = _side(n, ol)
        for i in torch.nonzero(rs & ~drop).flatten().tolist():
            e = side + int(sl_[i]) * (ol + 5)
            o[i, :ol + 4] = f[e + 1:e + 1 + ol + 4]
            o[i, 2 * ol + 4:] = f[e + 1 + ol:e + 1 + ol + 4]
    out[:nrows] = full[row0:row0 + nrows]
    return out


_LIVE_XCHG = _weakref.WeakSet()     # native exchanges not closed yet: destroyed at exit, before the runtime unloads
XCHG_MAX_COPIES = 64                 # host count buffers one native exchange tracks (cf2_xchg_copy_sync)


class _NativeCopy:
    """The completion of a look-ahead count copy the native exchange made into a host buffer
    (the event the library records after it: cf2_xchg_copy_sync).  A torch event per copy plus a
    stream wait cost ~8 us of host time per copy."""
    __slots__ = ("lib", "x", "ptr")

    def __init__(self, lib, x, ptr: int):
        self.lib, self.x, self.ptr = lib, x, ptr

    def synchronize(self):
        from . import _native
        _native.check(self.lib.cf2_xchg_copy_sync(self.x, self.ptr), "cf2_xchg_copy_sync")


def _raw_stream(device) -> int:
    """The current HIP stream of `device` as a raw handle (torch.cuda.current_stream(d).cuda_stream
    without building a Stream object: ~0.2 instead of ~1.9 us per call)."""
    import torch
    return torch._C._cuda_getCurrentRawStream(device.index if device.index is not None else torch.cuda.current_device())


def _close_live_exchanges():
    for g in list(_LIVE_XCHG):
        g.close()


def _pg_device(group, device):
    """Where the process group's collectives take their tensors: the GPU over RCCL, the host over gloo."""
    import torch.distributed as dist
    return device if dist.get_backend(group) == "nccl" else "cpu"


def _agree(ok: bool, group, device) -> bool:
    """True on every rank iff ok on every rank (all_reduce MIN over the group)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=_pg_device(group, device))
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _native_exchange(lib, group, world: int, depth: int, device, rccl_path: str | None = None):
    """The RCCL communicator of cf2_xchg_* for this group, created on `device` (collective: every
    rank calls it).  Every stage ends with an agreement over the process group, so a failure on one
    rank makes every rank fall back together (returns None) instead of leaving the others blocked
    in the id broadcast or in the communicator's rendezvous.  PyTorch's own RCCL instance where it
    ships one (or the library at rccl_path); rank 0's id broadcast over the process group."""
    import ctypes
    import torch
    import torch.distributed as dist
    from . import _native
    path = rccl_path or os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    ok = lib.cf2_xchg_bind(path.encode() if os.path.exists(path) else None) == 0
    rank = dist.get_rank(group)
    idb = (ctypes.c_uint8 * 128)()
    if ok and rank == 0:
        ok = lib.cf2_xchg_unique_id(idb, 128) == 0
    if not _agree(ok, group, device):
        return None
    t = torch.tensor(list(bytes(idb)), dtype=torch.uint8, device=_pg_device(group, device))
    dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    idb = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(t.cpu().tolist()))
    h = ctypes.c_void_p()
    with torch.cuda.device(device):
        st = lib.cf2_xchg_create(idb, 128, world, rank, depth, ctypes.byref(h))
    if not _agree(st == 0, group, device):
        if st == 0:
            _native.check(lib.cf2_xchg_destroy(h), "cf2_xchg_destroy")
        return None
    return h


class PipelinedObsGather:
    """Per-step all-gather of the observation slab ("RCCL all-gather over
    xGMI only for the returned observation tensor"), overlapped with the next env-steps.

    Env-step k writes ``buffer()`` (and, with ``delta``, ``done_buffer()``) on the current stream;
    ``publish()`` starts the exchange of that step on a side stream, so it runs while step k + 1
    computes.  Before an env-step overwrites a buffer, the current stream (not the host) waits for
    the exchange that read it.  On gloo (the CPU rehearsal of the multi-rank path) the exchange
    stages through the host and completes inside ``publish()``.

    delta=False: every step all-gathers the whole [n, D] slab of every rank; ``publish()`` returns
    the [world * n, D] slab (complete after ``drain()``; valid until the publish of step k + depth).

    delta=True: every step all-gathers only what a receiver cannot rebuild (cf2_obs_pack: o_k of
    every env, a reset bitmap, the reset rows' o_0 and action part for up to the step's capacity),
    and every receiver only advances the envs' ages (cf2_obs_consume): nothing is rebuilt per step.
    ``rows(act, act_prev, act_prev2)`` materialises rows of the latest published step on request
    (cf2_obs_rows) from the gathered buffers of that step and the one before and the actions of
    the last three steps ([world * n, 4], the policy's own outputs); they are valid until the next
    publish / run.  ``start(obs)`` gathers the observations of a reset of every env in full first.
    The native exchange runs over RCCL process groups; ``rccl_path`` binds it to another library
    with RCCL's four entry points instead (cf2_xchg_bind), also under a gloo group (the tests'
    world-size-2 stand-in on one GPU).
    The side capacity of step k is ``cap`` (the crash budget, default_cap) plus the time-outs the
    step can have at most (max_steps: the env's TimeLimit; the receivers count the envs that reach
    max_steps - lookahead, every rank the same, and the host reads the count ``lookahead`` steps
    later), so synchronised time-outs never overflow.  Over RCCL with the native exchange,
    ``run(env, act_ptrs, steps)`` takes ``steps`` env-steps of ``env`` in batches of ``unit``: the
    env-steps (the pack fused in) back to back on the current stream, one all-gather and one consume
    per batch on the exchange stream (cf2_xchg_run).  Buffers rotate over ``depth`` regions, one per
    publish / batch.  Shards must be equal (ValueError otherwise)."""

    def __init__(self, n: int, obs_dim: int, device, group=None, depth: int = 2, delta: bool = False,
                 cap: int | None = None, max_steps: int = 0, lookahead: int | None = None, unit: int = RUN_UNIT,
                 rccl_path: str | None = None):
        import torch
        import torch.distributed as dist
        if not 2 <= int(depth) <= 8:
            raise ValueError("PipelinedObsGather: depth must be 2..8 (a step's rows are built from the gathered "
                             "buffers of that step and the one before)")
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.nccl = dist.get_backend(group) == "nccl"
        sizes = exchange_sizes(n, group)
        if len(set(sizes)) != 1:
            raise ValueError(f"PipelinedObsGather needs equal shards, got {sizes}")
        self.n, self.od, self.ol = int(n), int(obs_dim), int(obs_dim) // 2 - 4
        self.depth = int(depth)
        self.delta = bool(delta)
        self.device = torch.device(device)
        cuda = self.device.type == "cuda"
        self.obs = [torch.empty(n, obs_dim, device=device) for _ in range(self.depth)]
        native_ok = cuda and (self.nccl or (self.delta and rccl_path is not None))
        self.comm = torch.cuda.Stream(device=self.device) if native_ok else None
        self.k = 0
        self.started = not self.delta
        self.bytes_sent = 0                  # this rank's contribution to every gather since start()
        self.steps_sent = 0
        self._xchg = None
        self._lib = None
        if not self.delta:
            self.out = [torch.empty(self.world * n, obs_dim, device=device) for _ in range(self.depth)]
            self._free = [None] * self.depth
            return
        self.unit = int(unit)
        if not 1 <= self.unit <= 64:
            raise ValueError("unit must be 1..64 env-steps")
        self.L = 3 * self.unit if lookahead is None else int(lookahead)
        # the host reads step s's count when it sizes step s + L: an eager copy is made every
        # PRED_BATCH steps, a run() copy after each batch, and a batch's capacity needs the counts of
        # its steps - L, which the copy of a batch at least one batch earlier than the last one in
        # flight holds
        if self.L < max(PRED_BATCH, 2 * self.unit + 1):
            raise ValueError(f"lookahead must be >= max({PRED_BATCH}, 2 * unit + 1) = {max(PRED_BATCH, 2 * self.unit + 1)}")
        self.cap = default_cap(n) if cap is None else int(cap)
        self.max_steps = int(max_steps)
        self.watch = self.max_steps - self.L if self.max_steps > self.L else NO_WATCH
        # ring of per-step counts: a consume writes its steps' rows and zeroes the ZERO_AHEAD rows after
        # them, so a host copy made after step e holds the counts of steps e - npred + ZERO_AHEAD + 1 .. e
        self.npred = max(self.L + 2 * ZERO_AHEAD + 1, NPRED_MIN)
        self.done = [torch.zeros(n, dtype=torch.uint8, device=device) for _ in range(self.depth)]
        self.age = torch.zeros(self.world * n, dtype=torch.int16 if cuda else torch.int32, device=device)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
        self.pred = torch.zeros(self.npred, self.world, dtype=torch.int32, device=device)
        npool = self.L // min(PRED_BATCH, self.unit) + 3
        if npool > XCHG_MAX_COPIES:
            raise ValueError(f"lookahead {self.L} needs {npool} count buffers, more than {XCHG_MAX_COPIES}")
        self._pred_pool = [torch.zeros(self.npred, self.world, dtype=torch.int32, pin_memory=cuda) for _ in range(npool)]
        self._pred_ptrs = [b.data_ptr() for b in self._pred_pool]
        self._pool_i = 0
        self._copies = []                    # (last step e covered, host buffer, event or None) in issue order
        self._counts = {}                    # step -> max count over ranks (the look-ahead window)
        self._where = {}                     # step -> (region, slot in its batch, batch size, capacity)
        self._region = 0                     # publishes / batches so far (their region: % depth)
        self._start_rows = None
        self._batch = None                   # step(): [k0, nb, cap, region, steps issued] of the open batch
        self._words = {}                     # capacity -> packed words (bookkeeping cache)
        if self.comm is not None:
            from . import _native
            self._lib = _native.load()
            # the whole exchange natively on our own RCCL communicator (cf2_xchg_*), unless
            # CF2SIM_EXCHANGE=torch asks for the process group's all-gather between the launches
            if os.environ.get("CF2SIM_EXCHANGE", "native") == "native":
                self._xchg = _native_exchange(self._lib, group, self.world, self.depth, self.device, rccl_path)
                if self._xchg is None:
                    import warnings
                    warnings.warn("native exchange unavailable on some rank; using the process group's all-gather")
            if self._xchg is None and not self.nccl:
                self.comm = None             # a gloo group without the native exchange: via the host
        # buffers: `depth` regions, each the packed buffers of a batch of up to kmax steps; the side-slot
        # counters of every (region, slot) after them (csrc/cf2sim_exchange.hip, cf2_xchg_register)
        self.kmax = self.unit if self._xchg is not None else 1
        self.wmax = packed_words(n, self.ol, n)
        nslot = self.depth * self.kmax
        self.send = torch.zeros(nslot * (self.wmax + PACK_SCRATCH_WORDS), dtype=torch.int32, device=device)
        self.recv = torch.zeros(nslot * self.world * self.wmax, dtype=torch.int32, device=device)
        self._scr0 = nslot * self.wmax
        if self._xchg is not None:
            import ctypes
            from . import _native
            assert self._lib.cf2_xchg_send_words(n, self.ol, self.depth, self.kmax) == self.send.numel()
            assert self._lib.cf2_xchg_recv_words(n, self.ol, self.world, self.depth, self.kmax) == self.recv.numel()
            arr = lambda ts: (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])     # noqa: E731
            self._reg = [arr(self.obs), arr(self.done)]
            _native.check(self._lib.cf2_xchg_register(
                self._xchg, self.n, self.ol, int(self.watch) & 0xFFFFFFFF, self.kmax, *self._reg, self.send.data_ptr(),
                self.recv.data_ptr(), self.age.data_ptr(), self.overflow.data_ptr(), self.pred.data_ptr(), self.npred),
                "cf2_xchg_register")
            _LIVE_XCHG.add(self)
            if len(_LIVE_XCHG) == 1:
                import atexit
                atexit.register(_close_live_exchanges)
        elif self.comm is not None:
            E = torch.cuda.Event
            self._ev_free = [E() for _ in range(self.depth)]
            self._free_rec = [False] * self.depth
            self._ev_end = E()

    @property
    def exchange(self) -> str:
        """How a step's exchange runs: 'native' (cf2_xchg_* calls: per step, or batched through
        run()), 'torch' (launches and the process group's all-gather from Python), 'gloo' or
        'full'."""
        if not self.delta:
            return "full"
        if self.comm is None:
            return "gloo"
        return "native" if self._xchg is not None else "torch"

    def close(self):
        """Release the native exchange's communicator (also run at exit)."""
        x = getattr(self, "_xchg", None)
        if x is not None:
            import torch
            torch.cuda.synchronize(self.device)
            self._xchg = None
            _LIVE_XCHG.discard(self)
            from . import _native
            _native.check(self._lib.cf2_xchg_destroy(x), "cf2_xchg_destroy")

    def __del__(self):
        try:
            self.close()
        except Exception:       # interpreter shutdown: the runtime may be gone already
            pass

    @property
    def bytes_per_rank_per_step(self) -> int:
        """Bytes one rank contributed to the all-gather of one env-step (delta: the mean since
        start(); before any step, that of the base capacity)."""
        if not self.delta:
            return 4 * self.n * self.od
        if self.steps_sent:
            return self.bytes_sent / self.steps_sent
        return 4 * packed_words(self.n, self.ol, self.cap)

    def _stream(self):
        import torch
        return torch.cuda.current_stream(self.device)

    def _q(self) -> int:
        return self._region % self.depth

    def buffer(self):
        """The obs buffer the next env-step writes (the current stream first waits, on the device,
        for the exchange that last read it)."""
        if not self.delta:
            j = self.k % self.depth
            if self._free[j] is not None:
                self._stream().wait_event(self._free[j])
                self._free[j] = None
            return self.obs[j]
        q = self._q()
        if self._xchg is not None:
            self._lib.cf2_xchg_wait_free(self._xchg, q, self._stream().cuda_stream)
        elif self.comm is not None and self._free_rec[q]:
            self._stream().wait_event(self._ev_free[q])
        return self.obs[q]

    def done_buffer(self):
        """delta: the uint8 done (auto-reset) buffer the next env-step writes; call after buffer()."""
        return self.done[self._q()]

    def _gather(self, out, x):
        import torch.distributed as dist
        if self.nccl:
            dist.all_gather_into_tensor(out, x, group=self.group)
        else:
            gather_rows(x.reshape(1, -1), self.group, sizes=[1] * self.world, out=out.view(self.world, -1))

    def _send(self, q: int, s: int, words: int):
        off = q * self.kmax * self.wmax + s * words
        return self.send[off:off + words]

    def _scratch(self, q: int, s: int):
        off = self._scr0 + (q * self.kmax + s) * PACK_SCRATCH_WORDS
        return self.send[off:off + PACK_SCRATCH_WORDS]

    def _recv_at(self, where):
        """(tensor starting at rank 0's packed buffer, capacity, rank stride) of a step's location."""
        if where[0] == "start":
            return self._start_pk, 0, packed_words(self.n, self.ol, 0)
        q, s, nb, cap = where
        words = packed_words(self.n, self.ol, cap)
        off = q * self.world * self.kmax * self.wmax + s * words
        return self.recv[off:off + (self.world - 1) * nb * words + words], cap, nb * words

    def start(self, obs):
        """delta: gather the observations of a reset of every env ([n, D]) in full (returned: the
        [world * n, D] slab); every env's step count since its reset is 0 on every rank."""
        import torch
        if not self.delta:
            raise RuntimeError("start() is for the delta exchange")
        self.drain()
        full = torch.empty(self.world * self.n, self.od, device=self.device)
        if self.comm is not None:
            self.comm.wait_stream(self._stream())
            with torch.cuda.stream(self.comm):
                self._gather(full, obs.contiguous())
            self._stream().wait_stream(self.comm)
        else:
            self._gather(full, obs.contiguous())
        # "step -1": its o_k slab (the reset observations' o parts) is what step 0's rows take as
        # o_{k-1}; capacity 0, no resets
        w0, ol = packed_words(self.n, self.ol, 0), self.ol
        self._start_pk = torch.zeros(self.world * w0, dtype=torch.int32, device=self.device)
        pv = self._start_pk.view(self.world, w0)
        pv[:, 4:4 + self.n * ol].view(torch.float32).copy_(full[:, ol + 4:2 * ol + 4].reshape(self.world, -1))
        self.age.zero_()
        self.pred.zero_()
        self.send[self._scr0:].zero_()
        self._where = {-1: ("start",)}
        self._counts, self._copies = {}, []
        self._start_rows = full
        self.started = True
        self.k = 0
        return full

    # ---- time-out look-ahead ----
    def _next_pool(self):
        b = self._pred_pool[self._pool_i % len(self._pred_pool)]
        self._pool_i += 1
        return b

    def _next_pool_ptr(self):
        """(buffer, its address) of the next count buffer."""
        j = self._pool_i % len(self._pred_pool)
        self._pool_i += 1
        return self._pred_pool[j], self._pred_ptrs[j]

    def _count(self, s: int) -> int:
        """The look-ahead count of step s (max over ranks), from the first host copy made at or
        after step s (waiting for it on the host)."""
        if s in self._counts:
            return self._counts[s]
        while self._copies:
            e, buf, ev = self._copies.pop(0)
            if e < s:
                continue
            if ev is not None:
                ev.synchronize()
            lo = max(e - self.npred + ZERO_AHEAD + 1, 0)
            # one vectorised max over ranks per copy: a torch op per step cost ~3 us of host time
            # each, ~170 us per batch of 16 (tools/run_host_probe.py), more than the batch's launches
            mx = buf.numpy().max(axis=1).tolist()
            for t in range(lo, e + 1):
                if t not in self._counts:
                    self._counts[t] = mx[t % self.npred]
            for t in [t for t in self._counts if t < lo - self.npred]:
                del self._counts[t]
            break
        if s not in self._counts:
            raise RuntimeError(f"delta exchange: the time-out count of step {s} was never copied to the host")
        return self._counts[s]

    def step_cap(self, k: int) -> int:
        """Side capacity of env-step k (0-based since start()): the crash budget plus the time-outs
        that step can have at most."""
        if self.watch == NO_WATCH:
            return self.n if 0 < self.max_steps else self.cap
        if k < self.L:                       # before the first prediction: every env is k + 1 old
            t = self.n if k + 1 == self.max_steps else 0
        else:
            t = self._count(k - self.L)
        return min(self.n, self.cap + t)

    def _after(self, k0: int, nb: int, cap: int, q: int, copied: bool):
        """Bookkeeping after the exchange of steps k0 .. k0 + nb - 1 (region q) was issued."""
        import torch
        for s in range(nb):
            self._where[k0 + s] = (q, s, nb, cap)
        for t in [t for t in self._where if t < k0 + nb - 2]:
            del self._where[t]
        self._region += 1
        self.k = k0 + nb
        w = self._words.get(cap)
        if w is None:
            w = self._words[cap] = packed_words(self.n, self.ol, cap)
        self.bytes_sent += 4 * w * nb
        self.steps_sent += nb
        e = k0 + nb - 1
        if not copied and self.watch != NO_WATCH and self.k // PRED_BATCH != k0 // PRED_BATCH:
            # the count ring to the host every PRED_BATCH steps (read lookahead steps later)
            buf = self._next_pool()
            if self.pred.is_cuda:
                # on a side stream behind the exchange: the env stream does not wait for it, and the
                # native copy (device stores into the pinned buffer) does not hold this thread
                s = self._side_stream()
                if self._xchg is not None:
                    from . import _native
                    _native.check(self._lib.cf2_xchg_pred_to_host(self._xchg, buf.data_ptr(), s.cuda_stream),
                                  "cf2_xchg_pred_to_host")
                else:
                    if self.comm is not None:
                        s.wait_event(self._ev_end)
                    else:
                        s.wait_stream(self._stream())
                    with torch.cuda.stream(s):
                        buf.copy_(self.pred, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s)
            else:
                buf.copy_(self.pred)
                ev = None
            self._copies.append((e, buf, ev))

    def publish(self):
        """Start the exchange of the buffer(s) the current env-step wrote.  Full rows: returns the
        slab it fills.  delta: returns the step's index (its rows: rows())."""
        import torch
        if not self.delta:
            j = self.k % self.depth
            out = self.out[j]
            if self.comm is not None:
                self.comm.wait_stream(self._stream())
                with torch.cuda.stream(self.comm):
                    torch.distributed.all_gather_into_tensor(out, self.obs[j], group=self.group)
                    ev = torch.cuda.Event()
                    ev.record(self.comm)
                self._free[j] = ev
            else:
                gather_rows(self.obs[j], self.group, sizes=[self.n] * self.world, out=out)
            self.k += 1
            return out
        if not self.started:
            raise RuntimeError("delta exchange: call start(reset observations) first")
        self.flush()
        k, q = self.k, self._q()
        cap = self.step_cap(k)
        words = packed_words(self.n, self.ol, cap)
        send = self._send(q, 0, words)
        recv = self.recv[q * self.world * self.kmax * self.wmax:][:self.world * words]
        qn = (self._region + 1) % self.depth
        w = self.watch != NO_WATCH
        ps = self.pred[k % self.npred] if w else None
        pn = self.pred[(k + 1) % self.npred] if w else None
        if self._xchg is not None:
            from . import _native
            _native.check(self._lib.cf2_xchg_publish(self._xchg, k, cap, q, self._stream().cuda_stream),
                          "cf2_xchg_publish")
        elif self.comm is not None:
            pack_obs(self.obs[q], self.done[q], cap, out=send, scratch=self._scratch(q, 0),
                     next_scratch=self._scratch(qn, 0))
            comm = self.comm
            comm.wait_stream(self._stream())
            with torch.cuda.stream(comm):
                torch.distributed.all_gather_into_tensor(recv, send, group=self.group)
                self._ev_free[q].record(comm)          # the region's buffers are free after the all-gather
                self._free_rec[q] = True
                consume_obs(recv, self.world, self.n, self.ol, cap, self.age, self.overflow, self.watch, ps, pn)
                self._ev_end.record(comm)
        else:
            cuda = send.is_cuda
            pack_obs(self.obs[q], self.done[q], cap, out=send, scratch=self._scratch(q, 0) if cuda else None,
                     next_scratch=self._scratch(qn, 0) if cuda else None)
            if recv.is_cuda:                       # gloo with GPU tensors: via the host
                host = gather_rows(send.cpu().reshape(1, -1), self.group, sizes=[1] * self.world)
                recv.copy_(host.reshape(-1))
            else:
                self._gather(recv, send)
            consume_obs(recv, self.world, self.n, self.ol, cap, self.age, self.overflow, self.watch, ps, pn)
        self._after(k, 1, cap, q, copied=False)
        return k

    def step_and_publish(self, env, act_ptr: int):
        """Native exchange: env-step k of `env` (this rank's shard; act_ptr its [n, 4] actions, a raw
        device pointer, not checked) with its pack fused in, then that step's exchange, in one C call
        (cf2_xchg_env_step: what buffer() + env.step_raw(...) + publish() do; every PRED_BATCH-th
        step it also copies the look-ahead counts to a host buffer).  The exchange runs inline on the
        current stream: the caller wants each step's rows before the next step, so there is nothing
        to overlap, and the fork / join events it saves are host time of the eager loop.  Returns k."""
        x = self._xchg
        if x is None:
            raise RuntimeError("step_and_publish needs the native exchange (RCCL, delta=True)")
        if not self.started:
            raise RuntimeError("delta exchange: call start(reset observations) first")
        if env.num_envs != self.n or env.obs_dim != self.od:
            raise ValueError("step_and_publish: the env's shard does not match the exchange's layout")
        if self._batch is not None:
            self.flush()
        k = self.k
        q = self._region % self.depth
        cap = self.step_cap(k)
        rew, trunc, cost, level = env._raw_step_outputs()
        sp = _raw_stream(self.device)
        lib = self._lib
        if self.watch != NO_WATCH and (k + 1) // PRED_BATCH != k // PRED_BATCH:
            buf, ptr = self._next_pool_ptr()
            st = lib.cf2_xchg_env_step(x, env._ctx, k, cap, q, act_ptr, rew, trunc, cost, level, ptr, sp)
            if st == 0:
                self._copies.append((k, buf, _NativeCopy(lib, x, ptr)))
        else:
            st = lib.cf2_xchg_env_step(x, env._ctx, k, cap, q, act_ptr, rew, trunc, cost, level, None, sp)
        if st != 0:
            from . import _native
            _native.check(st, "cf2_xchg_env_step")
        self._after(k, 1, cap, q, copied=True)
        return k

    def run(self, env, act_ptrs, steps: int) -> int:
        """Native exchange: `steps` env-steps of `env` (this rank's shard), the actions of step k at
        act_ptrs[k % len(act_ptrs)] (raw device pointers to [n, 4] float32, e.g. a ring the policy
        fills ahead, or a synthetic rollout's), in batches of `unit` aligned to multiples of it: a
        batch's env-steps (the pack fused in) back to back on the current stream, then one
        all-gather and one consume of the batch on the exchange stream, which run while the next
        batch steps (cf2_xchg_run).  A batch's side capacity is the largest of its steps'.  Returns
        the index of the last step (its rows: rows())."""
        import ctypes
        import torch
        if self._xchg is None:
            raise RuntimeError("run needs the native exchange (RCCL, delta=True)")
        if not self.started:
            raise RuntimeError("delta exchange: call start(reset observations) first")
        if env.num_envs != self.n or env.obs_dim != self.od:
            raise ValueError("run: the env's shard does not match the exchange's layout")
        nact = len(act_ptrs)
        if nact < 1:
            raise ValueError("run: at least one action buffer")
        self.flush()
        arr = (ctypes.c_void_p * nact)(*act_ptrs)
        rew, trunc, cost, level = env._raw_step_outputs()
        # the batches run on a stream of the exchange's own, ordered after the caller's stream and
        # before it again on return.  Issued on the null stream (torch's default) each batch's first
        # env-step waited for the previous batch's whole exchange (17.2 us per env-step at 32 768
        # envs, 14.3 on a pool stream: tools/xchg_run_probe.py --own-stream, gpurun_out/r05k)
        cur = self._stream()
        s = self._run_stream()
        s.wait_stream(cur)
        w = self.watch != NO_WATCH
        done = 0
        while done < steps:
            k0, q = self.k, self._q()
            nb = min(self.unit - k0 % self.unit, steps - done)
            cap = max(self.step_cap(k) for k in range(k0, k0 + nb))
            buf = self._next_pool() if w else None
            st = self._lib.cf2_xchg_run(self._xchg, env._ctx, k0, nb, cap, q, arr, nact, rew, trunc, cost, level,
                                        buf.data_ptr() if w else None, s.cuda_stream)
            if st != 0:
                from . import _native
                _native.check(st, "cf2_xchg_run")
            if w:
                # the batch's count copy ends on the exchange stream with an event of the library's,
                # which the host synchronises on when it reads the counts
                self._copies.append((k0 + nb - 1, buf, _NativeCopy(self._lib, self._xchg, buf.data_ptr())))
            self._after(k0, nb, cap, q, copied=True)
            done += nb
        cur.wait_stream(s)
        return self.k - 1

    def step(self, env, act_ptr: int) -> int:
        """Native exchange, a policy in the loop: env-step k of `env` (this rank's shard; act_ptr its
        [n, 4] actions, e.g. the policy's output on local_obs() of the step before) with its pack
        fused in, on the current stream.  The exchange runs per batch of `unit` steps aligned to
        multiples of it (cf2_xchg_begin / cf2_xchg_step / cf2_xchg_end: the same launches as run(),
        with the actions given one step at a time), so the gathered rows of a step are available
        once its batch is exchanged: at the batch's end or at flush().  Collective: every rank calls
        it for every env-step.  Returns k.  For the best overlap call it from a non-default stream
        (on the null stream a batch's first env-step waits for the previous batch's exchange)."""
        import torch
        from . import _native
        if self._xchg is None:
            raise RuntimeError("step needs the native exchange (RCCL, delta=True)")
        if not self.started:
            raise RuntimeError("delta exchange: call start(reset observations) first")
        if env.num_envs != self.n or env.obs_dim != self.od:
            raise ValueError("step: the env's shard does not match the exchange's layout")
        sp = torch.cuda.current_stream(self.device).cuda_stream
        if self._batch is None:
            k0, q = self.k, self._q()
            nb = self.unit - k0 % self.unit
            cap = max(self.step_cap(k) for k in range(k0, k0 + nb))
            _native.check(self._lib.cf2_xchg_begin(self._xchg, cap, q, sp), "cf2_xchg_begin")
            self._batch = [k0, nb, cap, q, 0]
        b = self._batch
        rew, trunc, cost, level = env._raw_step_outputs()
        _native.check(self._lib.cf2_xchg_step(self._xchg, env._ctx, act_ptr, rew, trunc, cost, level, sp),
                      "cf2_xchg_step")
        b[4] += 1
        k = b[0] + b[4] - 1
        if b[4] == b[1]:
            self.flush()
        return k

    def flush(self):
        """Exchange the env-steps step() has issued since the last exchange (collective: every rank
        calls it at the same step).  A no-op when there are none."""
        import torch
        b = self._batch
        if b is None:
            return
        from . import _native
        self._batch = None
        k0, nb, cap, q, s = b
        w = self.watch != NO_WATCH
        buf = self._next_pool() if w else None
        _native.check(self._lib.cf2_xchg_end(self._xchg, k0, buf.data_ptr() if w else None,
                                             torch.cuda.current_stream(self.device).cuda_stream), "cf2_xchg_end")
        if w:
            self._copies.append((k0 + s - 1, buf, _NativeCopy(self._lib, self._xchg, buf.data_ptr())))
        self._after(k0, s, cap, q, copied=True)

    def local_obs(self):
        """This rank's observation rows [n, D] of the latest env-step (step(), run(), step_and_publish
        or the caller's env-step into buffer()), before or after their exchange: what a policy in the
        loop acts on.  The done flags of that step: local_done()."""
        if not self.delta or not self.started:
            raise RuntimeError("local_obs(): a delta exchange after start()")
        if self._batch is not None:
            return self.obs[self._batch[3]]
        if self.k > 0:
            return self.obs[self._where[self.k - 1][0]]
        return self._start_rows[self.rank * self.n:(self.rank + 1) * self.n]

    def local_done(self):
        if not self.delta or not self.started:
            raise RuntimeError("local_done(): a delta exchange after start()")
        if self._batch is not None:
            return self.done[self._batch[3]]
        return self.done[self._where[self.k - 1][0]] if self.k > 0 else None

    def _run_stream(self):
        import torch
        if getattr(self, "_rs", None) is None:
            self._rs = torch.cuda.Stream(device=self.device)
        return self._rs

    def _side_stream(self):
        import torch
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.device)
        return self._side

    def rows(self, act, act_prev, act_prev2, out=None, row0: int = 0, nrows: int | None = None):
        """delta: rows [row0, row0 + nrows) (default: all world * n) of the latest published step's
        observation slab, materialised on the current stream (cf2_obs_rows) after that step's
        exchange: act / act_prev / act_prev2 = the actions of that step and of the two before it
        ([world * n, 4]; at the first steps after start() pass the earliest ones again).  Valid until
        the next publish / run.  Before any step: the slab start() gathered."""
        if not self.delta:
            raise RuntimeError("rows() is for the delta exchange")
        if self._batch is not None:
            raise RuntimeError("rows(): step() has env-steps not yet exchanged; call flush() on every rank first")
        k = self.k - 1
        N = self.world * self.n
        nrows = N - row0 if nrows is None else int(nrows)
        if k < 0:
            res = self._start_rows[row0:row0 + nrows]
            if out is not None:
                out.copy_(res)
                return out
            return res
        self.drain()
        cur, cap, st = self._recv_at(self._where[k])
        prev, cap_p, st_p = self._recv_at(self._where[k - 1])
        return obs_rows(cur, cap, prev, cap_p, self.world, self.n, self.ol, self.age, act, act_prev, act_prev2,
                        out=out, row0=row0, nrows=nrows, stride=st, stride_prev=st_p)

    def overflows(self) -> int:
        """delta: 64-env pack blocks whose resets found no side slot so far (host read)."""
        return int(self.overflow.item()) if self.delta else 0

    def drain(self):
        """Make the current stream wait for every exchange in flight."""
        s = self._stream() if self.device.type == "cuda" else None
        if s is None:
            return
        if self._xchg is not None:
            self._lib.cf2_xchg_wait(self._xchg, s.cuda_stream)
        elif self.comm is not None:
            s.wait_stream(self.comm)
        if not self.delta:
            self._free = [None] * self.depth


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
