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


# ---- delta observation exchange (csrc/cf2sim_exchange.hip has the protocol; cf2_obs_pack /
# cf2_obs_unpack run it on GPU tensors, the torch-op versions below on CPU tensors for the gloo
# rehearsal of the multi-rank path; both produce the same rows bit for bit) ----

PACK_BLOCK = 256      # envs per pack block: one block-table word each (the block's first side slot)


def _side(n: int, ol: int) -> int:
    """Word offset of the side entries: header, o_k rows, bitmap, block table."""
    return 4 + n * ol + (n + 31) // 32 + (n + PACK_BLOCK - 1) // PACK_BLOCK


def packed_words(n: int, ol: int, cap: int) -> int:
    """32-bit words of one rank's packed buffer (cf2_obs_packed_words)."""
    return (_side(n, ol) + cap * (ol + 5) + 3) & ~3


def default_cap(n: int) -> int:
    """Side-slab capacity: 7.5 % of the shard.  The bench workload ends 4.1 % of its episodes per
    env-step in steady state and 5.7 % at the synchronised-start peak (profiles/r02_reset_rate.json);
    a step that exceeds it marks the rows it could not send (NaN) and counts an overflow."""
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


def pack_obs(obs, reset, cap: int, out=None, clear_next=None):
    """One rank's packed buffer (int32 [packed_words]) from its step's obs rows [n, OD] and
    auto-reset flags [n] (uint8 or bool)."""
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
        # the kernel indexes by these sizes: check them on the host before the launch
        _need(obs.is_contiguous() and obs.dtype == torch.float32, "obs must be contiguous float32 [n, OD]")
        _need(reset.numel() >= n and reset.is_cuda, "reset needs n flags on the GPU")
        _need(out.dtype == torch.int32 and out.is_contiguous() and out.numel() >= words and out.is_cuda,
              f"out needs {words} int32 words on the GPU")
        _need(clear_next is None or (clear_next.is_cuda and clear_next.numel() >= 1), "clear_next needs 1 word")
        r8 = reset if reset.dtype == torch.uint8 else reset.to(torch.uint8)
        _native.check(lib.cf2_obs_pack(obs.data_ptr(), r8.contiguous().data_ptr(), n, ol, cap, out.data_ptr(),
                                       _native.ptr(clear_next), torch.cuda.current_stream(obs.device).cuda_stream),
                      "cf2_obs_pack")
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
    idx = torch.nonzero(r).flatten()
    out[0], out[1], out[2], out[3] = int(idx.numel()), n, ol, cap
    # block table: the first side slot of each pack block's resets (blocks in env order here; the
    # GPU kernel hands slots out per block in any order, so only the slots differ, not the rows)
    nblk = (n + PACK_BLOCK - 1) // PACK_BLOCK
    per_blk = torch.zeros(nblk, dtype=torch.int64)
    per_blk.index_add_(0, idx // PACK_BLOCK, torch.ones_like(idx))
    out[4 + n * ol + nb:4 + n * ol + nb + nblk] = (torch.cumsum(per_blk, 0) - per_blk).to(torch.int32)
    side = _side(n, ol)
    for s, i in enumerate(idx[:cap].tolist()):
        e = side + s * (ol + 5)
        out[e] = i
        f[e + 1:e + 1 + ol + 4] = obs[i, :ol + 4]
    if clear_next is not None:
        clear_next.zero_()
    return out


NO_WATCH = 0xFFFFFFFF
PRED_BATCH = 4          # RCCL delta path: time-out counts copied to the host every 4 steps (< lookahead)

_LIVE_XCHG = set()      # native exchanges not closed yet: destroyed at exit, before the runtime unloads


def _close_live_exchanges():
    for g in list(_LIVE_XCHG):
        g.close()


def _native_exchange(lib, group, world: int, depth: int, device):
    """The RCCL communicator of cf2_xchg_* for this group (collective: every rank calls it): rank
    0's id broadcast over the process group; PyTorch's own RCCL instance where it ships one."""
    import ctypes
    import torch
    import torch.distributed as dist
    from . import _native
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    _native.check(lib.cf2_xchg_bind(path.encode() if os.path.exists(path) else None), "cf2_xchg_bind")
    idb = (ctypes.c_uint8 * 128)()
    rank = dist.get_rank(group)
    if rank == 0:
        _native.check(lib.cf2_xchg_unique_id(idb, 128), "cf2_xchg_unique_id")
    t = torch.tensor(list(bytes(idb)), dtype=torch.uint8, device=device)
    dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    idb = (ctypes.c_uint8 * 128).from_buffer_copy(bytes(t.cpu().tolist()))
    h = ctypes.c_void_p()
    _native.check(lib.cf2_xchg_create(idb, 128, world, rank, depth, ctypes.byref(h)), "cf2_xchg_create")
    return h


def unpack_obs(recv, world: int, n: int, ol: int, cap: int, act, act_prev, age, slab_prev, slab, overflow=None,
               watch_age: int = NO_WATCH, pred=None, pred_next=None):
    """Rebuild every rank's rows [world n, OD] into `slab` from the gathered packed buffers
    (int32 [world * packed_words(n, ol, cap)]), the previous slab, the step's actions and the
    previous step's (act, act_prev: [world n, 4]); age (steps since reset; int16 storage of a
    uint16 on GPUs, int32 on the CPU, [world n]) is updated in place.  Envs whose new age equals
    watch_age are counted per rank into pred ([world]); pred_next is zeroed."""
    import torch
    if recv.is_cuda:
        from . import _native
        lib = _native.load()
        # the kernels index by these sizes: check them on the host before the launch
        N, od = world * n, 2 * (ol + 4)
        _need(recv.dtype == torch.int32 and recv.is_contiguous() and recv.numel() >= world * packed_words(n, ol, cap),
              "recv needs world * packed_words int32 words")
        _need(age.dtype == torch.int16 and age.is_contiguous() and age.numel() >= N and age.is_cuda,
              "age must be int16 (uint16 storage) [world * n] on the GPU")
        for name, t, cols in (("act", act, 4), ("act_prev", act_prev, 4), ("slab_prev", slab_prev, od), ("slab", slab, od)):
            _need(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() >= N * cols,
                  f"{name} must be contiguous float32 [world * n, {cols}] on the GPU")
        for name, t, k in (("overflow", overflow, 1), ("pred", pred, world), ("pred_next", pred_next, world)):
            _need(t is None or (t.is_cuda and t.dtype == torch.int32 and t.numel() >= k), f"{name} needs {k} int32")
        _native.check(lib.cf2_obs_unpack(recv.data_ptr(), world, n, ol, cap, act.data_ptr(), act_prev.data_ptr(),
                                         age.data_ptr(), slab_prev.data_ptr(), slab.data_ptr(), _native.ptr(overflow),
                                         int(watch_age) & 0xFFFFFFFF, _native.ptr(pred), _native.ptr(pred_next),
                                         torch.cuda.current_stream(recv.device).cuda_stream), "cf2_obs_unpack")
        return slab
    words = packed_words(n, ol, cap)
    rv = recv[:world * words].reshape(world, words)
    nan = float("nan")
    if pred_next is not None:
        pred_next.zero_()
    for r in range(world):
        pk = rv[r]
        f = pk.view(torch.float32)
        ok = f[4:4 + n * ol].view(n, ol)
        rs = _bits_to_mask(pk[4 + n * ol:4 + n * ol + (n + 31) // 32], n)
        sl = slice(r * n, (r + 1) * n)
        prev, out = slab_prev[sl], slab[sl]
        a = torch.clamp(age[sl].to(torch.int64) + 1, max=0xFFFF)
        out[:, :ol] = prev[:, ol + 4:2 * ol + 4]
        out[:, ol:ol + 4] = torch.where((a >= 3)[:, None], prev[:, 2 * ol + 4:], act[sl])
        out[:, ol + 4:2 * ol + 4] = ok
        out[:, 2 * ol + 4:] = torch.where((a == 1)[:, None], act[sl], act_prev[sl])
        cnt = int(pk[0])
        if cnt > cap:
            out[rs, :ol + 4] = nan
            out[rs, 2 * ol + 4:] = nan
            if overflow is not None:
                overflow += 1
        else:
            side = _side(n, ol)
            for s in range(cnt):
                e = side + s * (ol + 5)
                i = int(pk[e])
                out[i, :ol + 4] = f[e + 1:e + 1 + ol + 4]
                out[i, 2 * ol + 4:] = f[e + 1 + ol:e + 1 + ol + 4]
        new = torch.where(rs, torch.zeros_like(a), a)
        age[sl] = new.to(age.dtype)
        if pred is not None:
            pred[r] += int((new == watch_age).sum())
    return slab


class PipelinedObsGather:
    """Per-step all-gather of the observation slab ("RCCL all-gather over
    xGMI only for the returned observation tensor"), overlapped with the next env-step.

    Env-step k writes ``buffer()`` (and, with ``delta``, ``done_buffer()``) on the compute stream;
    ``publish()`` starts the exchange of that step on a side stream, so it runs while step k+1
    computes.  Before step k + depth overwrites a buffer, the compute stream (not the host) waits for
    the exchange step that read it.  ``publish()`` returns the [world * n, D] slab of step k; it is
    complete once ``drain()`` returned (or after ``ready()`` on any stream) and stays valid until
    the publish of step k + 2.  On gloo (the CPU rehearsal of the multi-rank path) the exchange
    stages through the host and completes inside ``publish()``.

    delta=False: every step all-gathers the whole [n, D] slab of every rank.
    delta=True: every step all-gathers only what a receiver cannot rebuild (cf2_obs_pack: o_k of
    every env, a reset bitmap, the reset rows' o_0 and action part for up to ``cap`` resets) and
    every rank rebuilds the full slab from its previous one and the actions (cf2_obs_unpack): the
    actions of step k and k - 1 for every env ([world * n, 4], the policy's own outputs) are
    arguments of ``publish``.  ``start(obs)`` gathers the observations of a reset of every env in
    full first.  The side capacity of a step is ``cap`` (the crash budget, default_cap) plus the
    time-outs that step can have at most (max_steps: the env's TimeLimit; the receivers count the
    envs that reach max_steps - lookahead, every rank the same, and the host reads the count
    ``lookahead`` steps later), so synchronised time-outs never overflow.  Shards must be equal
    (ValueError otherwise)."""

    def __init__(self, n: int, obs_dim: int, device, group=None, depth: int = 2, delta: bool = False,
                 cap: int | None = None, max_steps: int = 0, lookahead: int = 8):
        import torch
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
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
        self.comm = torch.cuda.Stream(device=self.device) if (self.nccl and cuda) else None
        # the rebuild runs on the exchange stream right after the all-gather: a third stream (the
        # rebuild of step k beside the all-gather of step k + 1) cost more host time per step than
        # it overlapped (the eager step is host-bound at the node shard: DESIGN.md section 6)
        self.free = [None] * self.depth      # events: the exchange of the step that used buffer j read it
        self.k = 0
        self.started = not self.delta
        self.bytes_sent = 0                  # this rank's contribution to every gather since start()
        self.steps_sent = 0
        if self.delta:
            self.cap = default_cap(n) if cap is None else int(cap)
            self.max_steps = int(max_steps)
            self.L = int(lookahead)
            # time-outs are predicted L steps ahead from the ages (watch age max_steps - L); a
            # TimeLimit of L steps or fewer is sent at full capacity instead
            self.watch = self.max_steps - self.L if self.max_steps > self.L else NO_WATCH
            wmax = packed_words(n, self.ol, n)
            self.done = [torch.zeros(n, dtype=torch.uint8, device=device) for _ in range(self.depth)]
            self.send = [torch.zeros(wmax, dtype=torch.int32, device=device) for _ in range(self.depth)]
            self.recv = [torch.empty(self.world * wmax, dtype=torch.int32, device=device) for _ in range(self.depth)]
            self.slab = [torch.zeros(self.world * n, obs_dim, device=device) for _ in range(2)]
            self.age = torch.zeros(self.world * n, dtype=torch.int16 if cuda else torch.int32, device=device)
            self.overflow = torch.zeros(1, dtype=torch.int32, device=device)
            self.pred = torch.zeros(self.L + 1, self.world, dtype=torch.int32, device=device)
            pin = cuda
            self.pred_host = torch.zeros(self.L + 1, self.world, dtype=torch.int32, pin_memory=pin)
            self.pred_ev = [None] * (self.L + 1)
        else:
            self.out = [torch.empty(self.world * n, obs_dim, device=device) for _ in range(self.depth)]
        # the RCCL delta path's per-step host work is kept small (the eager step is host-bound at
        # the node shard otherwise): buffers checked once here, raw pointers, reused events, views
        # cached per side capacity
        self._fast = self.delta and self.comm is not None
        self._xchg = None
        if self._fast:
            from . import _native
            self._lib = _native.load()
            E = torch.cuda.Event
            self._ev_fork = [E() for _ in range(self.depth)]
            self._ev_unp = [E() for _ in range(self.depth)]
            self._ev_pred = [E() for _ in range(self.L // PRED_BATCH + 3)]
            self._pred_batch = []                # (step, event) of the count-ring copies in flight
            self._views = {}
            self._comm_h = self.comm.cuda_stream
            self._p_send = [t.data_ptr() for t in self.send]
            self._p_recv = [t.data_ptr() for t in self.recv]
            self._p_obs = [t.data_ptr() for t in self.obs]
            self._p_done = [t.data_ptr() for t in self.done]
            self._p_slab = [t.data_ptr() for t in self.slab]
            self._p_pred = [self.pred[r].data_ptr() for r in range(self.L + 1)]
            # the whole step as one C call on our own RCCL communicator (cf2_xchg_step), unless
            # CF2SIM_EXCHANGE=torch asks for the process group's all-gather between the launches
            self._xchg = None
            if os.environ.get("CF2SIM_EXCHANGE", "native") == "native":
                if self.depth > 8:
                    raise ValueError("the native exchange keeps at most 8 buffers in flight")
                try:
                    self._xchg = _native_exchange(self._lib, group, self.world, self.depth, self.device)
                except _native.CF2Error as e:      # e.g. no RCCL library to bind: the torch path, said so
                    import warnings
                    warnings.warn(f"native exchange unavailable ({e}); using the process group's all-gather")
            if self._xchg is not None:
                self._p_age, self._p_ovf = self.age.data_ptr(), self.overflow.data_ptr()
                import ctypes
                arr = lambda ptrs: (ctypes.c_void_p * len(ptrs))(*ptrs)     # noqa: E731
                self._reg = [arr(self._p_obs), arr(self._p_done), arr(self._p_send), arr(self._p_recv),
                             arr(self._p_pred)]
                _native.check(self._lib.cf2_xchg_register(
                    self._xchg, self.n, self.ol, int(self.watch) & 0xFFFFFFFF, *self._reg[:4], self._p_slab[0],
                    self._p_slab[1], self._p_age, self._p_ovf, self._reg[4], self.L + 1,
                    self.pred_host.data_ptr() if self.watch != NO_WATCH else None, PRED_BATCH, len(self._ev_pred),
                    self._comm_h), "cf2_xchg_register")
                _LIVE_XCHG.add(self)
                if len(_LIVE_XCHG) == 1:
                    import atexit
                    atexit.register(_close_live_exchanges)

    @property
    def exchange(self) -> str:
        """How a step's exchange runs: 'native' (one cf2_xchg_step call), 'torch' (launches and the
        process group's all-gather from Python), 'gloo' or 'full'."""
        if not self.delta:
            return "full"
        if not self._fast:
            return "gloo"
        return "native" if self._xchg is not None else "torch"

    def close(self):
        """Release the native exchange's communicator (after drain(); also run at exit)."""
        x = getattr(self, "_xchg", None)
        if x is not None:
            import torch
            torch.cuda.synchronize(self.device)
            self._xchg = None
            _LIVE_XCHG.discard(self)
            from . import _native
            _native.check(self._lib.cf2_xchg_destroy(x), "cf2_xchg_destroy")

    @property
    def bytes_per_rank_per_step(self) -> int:
        """Bytes one rank contributed to the all-gather of one env-step (delta: the mean since
        start(); before any step, that of the base capacity)."""
        if not self.delta:
            return 4 * self.n * self.od
        if self.steps_sent:
            return self.bytes_sent / self.steps_sent
        return 4 * packed_words(self.n, self.ol, self.cap)

    def _wait_free(self, j):
        import torch
        f = self.free[j]
        if f is not None:
            if isinstance(f, torch.cuda.Event):
                torch.cuda.current_stream(self.device).wait_event(f)
            elif isinstance(f, int) and self._xchg is not None:     # native: the end event of slot f
                self._lib.cf2_xchg_wait(self._xchg, f, torch.cuda.current_stream(self.device).cuda_stream)
            self.free[j] = None

    def buffer(self):
        """The obs buffer env-step k writes (the current stream first waits, on the device, for the
        exchange of step k - depth, which read it)."""
        j = self.k % self.depth
        self._wait_free(j)
        return self.obs[j]

    def done_buffer(self):
        """delta: the uint8 done (auto-reset) buffer env-step k writes; call after buffer()."""
        return self.done[self.k % self.depth]

    def _gather(self, out, x):
        import torch.distributed as dist
        if self.nccl:
            dist.all_gather_into_tensor(out, x, group=self.group)
        else:
            gather_rows(x.reshape(1, -1), self.group, sizes=[1] * self.world, out=out.view(self.world, -1))

    def _run_on_comm(self, fn):
        import torch
        if self.comm is not None:
            self.comm.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.comm):
                return fn()
        return fn()

    def start(self, obs):
        """delta: gather the observations of a reset of every env ([n, D]) in full; every env's
        step count since its reset is 0 on every rank."""

        def run():
            self._gather(self.slab[1], obs.contiguous())
            self.age.zero_()
            self.pred.zero_()
            for s in self.send:
                s[:1].zero_()
        self._run_on_comm(run)
        self.pred_host.zero_()
        self.pred_ev = [None] * (self.L + 1)
        if self._fast:
            self._pred_batch = []
        self.started = True
        self.k = 0
        return self.slab[1]

    def step_cap(self, k: int) -> int:
        """Side capacity of env-step k (0-based since start()): the crash budget plus the time-outs
        that step can have at most."""
        if self.watch == NO_WATCH:
            return self.n if 0 < self.max_steps else self.cap
        if k < self.L:                       # before the first prediction: every env is k + 1 old
            t = self.n if k + 1 == self.max_steps else 0
        elif self._fast:
            # the first batch copy issued at or after step k - L (issued after that step's rebuild;
            # the slot is only cleared by the rebuild of step k, after this read)
            s = (k - self.L) % (self.L + 1)
            c, ev = next((c, e) for (c, e) in self._pred_batch if c >= k - self.L)
            if ev is None:                   # copied by cf2_xchg_env_step
                self._lib.cf2_xchg_pred_sync(self._xchg, c)
            else:
                ev.synchronize()
            t = int(self.pred_host[s].max())
        else:
            s = (k - self.L) % (self.L + 1)
            ev = self.pred_ev[s]
            if ev is not None:
                ev.synchronize()
            t = int(self.pred_host[s].max())
        return min(self.n, self.cap + t)

    def publish(self, act=None, act_prev=None):
        """Start the exchange of the buffer(s) the current env-step wrote; returns the slab it fills.
        delta: act / act_prev = the actions of this env-step and of the previous one for all
        world * n envs (unchanged until the slab is complete)."""
        import torch
        j = self.k % self.depth
        if not self.delta:
            def run():
                if self.nccl:
                    torch.distributed.all_gather_into_tensor(self.out[j], self.obs[j], group=self.group)
                else:
                    gather_rows(self.obs[j], self.group, sizes=[self.n] * self.world, out=self.out[j])
                if self.comm is not None:
                    ev = torch.cuda.Event()
                    ev.record(self.comm)
                    self.free[j] = ev
                return self.out[j]
            out = self._run_on_comm(run)
            self.k += 1
            return out
        if not self.started:
            raise RuntimeError("delta exchange: call start(reset observations) first")
        if act is None or act_prev is None:
            raise ValueError("delta exchange: publish needs the actions of this step and of the previous one")
        if self._fast:
            return self._publish_fast(act, act_prev)
        k = self.k
        cap = self.step_cap(k)
        words = packed_words(self.n, self.ol, cap)
        prev, cur = self.slab[(k + 1) % 2], self.slab[k % 2]
        ps, pn = k % (self.L + 1), (k + 1) % (self.L + 1)
        send, recv = self.send[j][:words], self.recv[j][:self.world * words]

        def unpack():
            watch = self.watch if self.watch != NO_WATCH else NO_WATCH
            unpack_obs(recv, self.world, self.n, self.ol, cap, act, act_prev, self.age, prev, cur, self.overflow,
                       watch, self.pred[ps] if watch != NO_WATCH else None,
                       self.pred[pn] if watch != NO_WATCH else None)
            if watch != NO_WATCH:
                self.pred_host[ps].copy_(self.pred[ps], non_blocking=True)
                if self.pred.is_cuda:             # the host reads it L steps later, after this event
                    pe = torch.cuda.Event()
                    pe.record(torch.cuda.current_stream(self.device))
                    self.pred_ev[ps] = pe
            if self.comm is not None:
                ev2 = torch.cuda.Event()
                ev2.record(torch.cuda.current_stream(self.device))
                self._ready = ev2

        def run():
            pack_obs(self.obs[j], self.done[j], cap, out=send, clear_next=self.send[(j + 1) % self.depth][:1])
            if self.comm is not None:
                ev = torch.cuda.Event()
                ev.record(self.comm)
                self.free[j] = ev
            if recv.is_cuda and not self.nccl:      # gloo with GPU tensors: via the host
                host = gather_rows(send.cpu().reshape(1, -1), self.group, sizes=[1] * self.world)
                recv.copy_(host.reshape(-1))
            else:
                self._gather(recv, send)
            unpack()
            return cur
        out = self._run_on_comm(run)
        self.bytes_sent += 4 * words
        self.steps_sent += 1
        self.k += 1
        return out

    def _publish_fast(self, act, act_prev):
        """publish() of the RCCL delta path: the general path's operations (pack, all-gather,
        rebuild, all on the exchange stream) with pre-checked buffers, raw pointers and reused
        events."""
        import torch
        import torch.distributed as dist
        k, j, D = self.k, self.k % self.depth, self.depth
        N = self.world * self.n
        if act.numel() < N * 4 or act_prev.numel() < N * 4 or not (act.is_cuda and act_prev.is_cuda):
            raise ValueError("delta exchange: act / act_prev must be [world * n, 4] on the GPU")
        cap = self.step_cap(k)
        key = (j, cap)
        v = self._views.get(key)
        if v is None:
            words = packed_words(self.n, self.ol, cap)
            v = self._views[key] = (words, self.send[j][:words], self.recv[j][:self.world * words])
        words, send, recv = v
        lib, comm = self._lib, self.comm
        watch = self.watch
        ps, pn = k % (self.L + 1), (k + 1) % (self.L + 1)
        w = watch != NO_WATCH
        if self._xchg is not None:
            # fork, pack, RCCL all-gather, rebuild and the end event of slot j: one C call
            st = lib.cf2_xchg_step(self._xchg, j, self._p_obs[j], self._p_done[j], self.n, self.ol, cap,
                                   self._p_send[j], self._p_send[(j + 1) % D], self._p_recv[j], act.data_ptr(),
                                   act_prev.data_ptr(), self._p_age, self._p_slab[(k + 1) % 2], self._p_slab[k % 2],
                                   self._p_ovf, int(watch) & 0xFFFFFFFF, self._p_pred[ps] if w else None,
                                   self._p_pred[pn] if w else None, torch.cuda.current_stream(self.device).cuda_stream,
                                   self._comm_h)
            if st != 0:
                from . import _native
                _native.check(st, "cf2_xchg_step")
        else:
            ef = self._ev_fork[j]
            ef.record(torch.cuda.current_stream(self.device))
            comm.wait_event(ef)
            st = lib.cf2_obs_pack(self._p_obs[j], self._p_done[j], self.n, self.ol, cap, self._p_send[j],
                                  self._p_send[(j + 1) % D], self._comm_h)
            if st != 0:
                from . import _native
                _native.check(st, "cf2_obs_pack")
            with torch.cuda.stream(comm):          # the synchronous call: 19 us of host time, async + wait 42 us
                dist.all_gather_into_tensor(recv, send, group=self.group)
            st = lib.cf2_obs_unpack(self._p_recv[j], self.world, self.n, self.ol, cap, act.data_ptr(),
                                    act_prev.data_ptr(), self.age.data_ptr(), self._p_slab[(k + 1) % 2],
                                    self._p_slab[k % 2], self.overflow.data_ptr(), int(watch) & 0xFFFFFFFF,
                                    self._p_pred[ps] if w else None, self._p_pred[pn] if w else None, self._comm_h)
            if st != 0:
                from . import _native
                _native.check(st, "cf2_obs_unpack")
        return self._published(k, j, words, w)

    def step_and_publish(self, env, act_ptr: int, act_all_ptr: int, act_prev_all_ptr: int):
        """Native exchange: env-step k of `env` (this rank's shard; act_ptr its [n, 4] actions) into
        the exchange's buffers, then that step's exchange, in one C call (cf2_xchg_env_step: what
        buffer() + env.step_raw(...) + publish(act_all, act_prev_all) do).  Raw device pointers,
        not checked (act_all / act_prev_all: [world * n, 4] float32, as publish() takes them).
        Returns the slab of step k."""
        import torch
        if self._xchg is None:
            raise RuntimeError("step_and_publish needs the native exchange (RCCL, delta=True)")
        if not self.started:
            raise RuntimeError("delta exchange: call start(reset observations) first")
        if env.num_envs != self.n or env.obs_dim != self.od:
            raise ValueError("step_and_publish: the env's shard does not match the exchange's layout")
        k, j = self.k, self.k % self.depth
        cap = self.step_cap(k)
        rew, trunc, cost, level = env._raw_step_outputs()
        st = self._lib.cf2_xchg_env_step(self._xchg, env._ctx, k, cap, act_ptr, act_all_ptr, act_prev_all_ptr, rew,
                                         trunc, cost, level, torch.cuda.current_stream(self.device).cuda_stream)
        if st != 0:
            from . import _native
            _native.check(st, "cf2_xchg_env_step")
        words = self._views.get(("w", cap))
        if words is None:
            words = self._views[("w", cap)] = packed_words(self.n, self.ol, cap)
        if self.watch != NO_WATCH and k % PRED_BATCH == 0:      # the C call copied the count ring
            self._pred_batch.append((k, None))
            if len(self._pred_batch) > len(self._ev_pred) - 1:
                self._pred_batch.pop(0)
        return self._published(k, j, words, False)

    def _published(self, k, j, words, w):
        """publish()'s bookkeeping after the exchange of step k (buffer slot j) was issued (w: copy
        the time-out count ring to the host at this step's batch boundary)."""
        import torch
        comm = self.comm
        if w and k % PRED_BATCH == 0:
            # the whole count ring to the host every PRED_BATCH steps: step_cap(k') reads the count of
            # step k' - L from the first batch copy at or after it (each is ~15 us of host work)
            with torch.cuda.stream(comm):
                self.pred_host.copy_(self.pred, non_blocking=True)
                pe = self._ev_pred[(k // PRED_BATCH) % len(self._ev_pred)]
                pe.record(comm)
            self._pred_batch.append((k, pe))
            if len(self._pred_batch) > len(self._ev_pred) - 1:
                self._pred_batch.pop(0)
        if self._xchg is not None:
            self._ready = j                    # the exchange that read obs / done buffer j ends at slot j
            self.free[j] = j
        else:
            eu = self._ev_unp[j]
            eu.record(comm)
            self._ready = eu
            self.free[j] = eu                  # the exchange that read obs / done buffer j ends here
        self.bytes_sent += 4 * words
        self.steps_sent += 1
        self.k += 1
        return self.slab[k % 2]

    def ready(self):
        """Make the current stream wait for the latest published slab."""
        import torch
        ev = getattr(self, "_ready", None)
        if isinstance(ev, int) and self._xchg is not None:
            self._lib.cf2_xchg_wait(self._xchg, ev, torch.cuda.current_stream(self.device).cuda_stream)
        elif ev is not None:
            torch.cuda.current_stream(self.device).wait_event(ev)

    def overflows(self) -> int:
        """delta: steps x ranks whose resets exceeded the side capacity so far (host read)."""
        return int(self.overflow.item()) if self.delta else 0

    def drain(self):
        """Make the current stream wait for every exchange in flight."""
        import torch
        if self.comm is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm)
        for j in range(self.depth):
            self.free[j] = None


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
