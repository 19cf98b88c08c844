"""BatchedCrazyflieEnv: N hover environments stepped by one fused HIP kernel per env-step.

This is the torch-ROCm face of the C ABI (include/cf2sim.h).  All tensors live on the
current HIP device; every call is asynchronous on torch's current stream; there is no CPU
fallback (construction fails loudly without a GPU or without libcf2sim.so).

Semantics per env follow the reference's single-process ``gym.make(id)`` env wrapped in
gym's ``TimeLimit(max_episode_steps=500)`` (phoenix_drone_simulation/__init__.py:8-109):
``step`` returns ``(obs, reward, done, info)`` where ``done = terminal or truncated``; envs
that finish are reset inside the same kernel (vector-env auto-reset) and their pre-reset
observation is returned in ``info['final_obs']`` when requested.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _native
from .config import CF2Config, DSTB_EXTERNAL, DSTB_HJ, build_config, obs_dim, spec_for_id
from .spaces import make_box


# where the reference keeps its HJ value tables, relative to its repository root (distur_gener.py:155)
REFERENCE_TABLE_DIR = "phoenix_drone_simulation/adversarial_generation/FasTrack_data"


def value_table_name(level: float) -> str:
    """The reference's file name of the value table for a disturbance level: distur_gener.py:155
    formats the level as Python prints it (0.0, 0.1, ..., 1.5, ...; Boltzmann() rounds to 1 decimal)."""
    return f"fastrack_{round(float(level), 1)}_15x15.npy"


def load_value_tables(source, cfg):
    """The HJ value tables an env of configuration ``cfg`` reads, as (V [T, 15**6] float32 numpy,
    table_of_level).  ``source``:
      * a directory holding ``fastrack_{level}_15x15.npy`` (the reference's FasTrack_data folder), or
        the reference's repository root (the files under ``REFERENCE_TABLE_DIR``);
      * a dict {level: array of 15**6 values};
      * an array [T, 15**6] / [15]*6 / [T, 15, ..., 15] (bound as given; one table = every level).
    Files are read with ``np.load(allow_pickle=False)`` (they are plain arrays; nothing in them is
    executed).  A fixed-level env needs the table of its level only; a Boltzmann-level env one per
    level of ``cfg.level_values`` (distur_gener loads ``fastrack_{level}`` per call)."""
    import os
    nl = int(cfg.num_levels)
    boltz = int(cfg.level_mode) == 1
    levels = [float(cfg.level_values[k]) for k in range(nl)] if boltz else [float(cfg.dstb_level)]
    if isinstance(source, (str, os.PathLike)):
        root = os.fspath(source)
        cand = [root, os.path.join(root, REFERENCE_TABLE_DIR)]
        tabs = {}
        for lv in levels:
            name = value_table_name(lv)
            path = next((os.path.join(d, name) for d in cand if os.path.isfile(os.path.join(d, name))), None)
            if path is None:
                raise FileNotFoundError(f"{name} not found in {root} or {os.path.join(root, REFERENCE_TABLE_DIR)}")
            tabs[round(lv, 1)] = np.load(path, allow_pickle=False)
        source = tabs
    if isinstance(source, dict):
        keys = {round(float(k), 1): v for k, v in source.items()}
        uniq, rows, tol = [], {}, []
        for lv in levels:
            k = round(lv, 1)
            if k not in keys:
                raise KeyError(f"no value table for level {k}")
            obj = id(keys[k])                 # levels given the same array share one row
            if obj not in rows:
                rows[obj] = len(uniq)
                uniq.append(np.asarray(keys[k], dtype=np.float32).reshape(-1))
            tol.append(rows[obj])
        V = np.stack(uniq)
        table_of_level = tol if boltz else [0] * nl
    else:
        V = np.asarray(source.cpu() if isinstance(source, torch.Tensor) else source, dtype=np.float32)
        V = V.reshape(-1, 15 ** 6) if V.size % 15 ** 6 == 0 else V
        table_of_level = None
    if V.ndim != 2 or V.shape[1] != 15 ** 6:
        raise ValueError("HJ value tables must be 15^6 grids")
    return np.ascontiguousarray(V), table_of_level


def _check_buf(t, name, shape, dtype, device, align=4):
    """Raise ValueError unless t is a contiguous `dtype` tensor of `shape` on `device` whose data
    pointer is `align`-byte aligned (the kernel reads and writes these buffers with no bounds
    information of its own)."""
    if t is None:
        return
    if not isinstance(t, torch.Tensor):
        raise ValueError(f"{name} must be a torch tensor")
    if t.device != device:
        raise ValueError(f"{name} must be on {device}, got {t.device}")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if tuple(t.shape) != tuple(shape):
        raise ValueError(f"{name} must have shape {tuple(shape)}, got {tuple(t.shape)}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.data_ptr() % align:
        raise ValueError(f"{name} must be {align}-byte aligned")


class BatchedCrazyflieEnv:
    def __init__(self, env_id: str, num_envs: int, seed: int = 0, device=None, env_id_offset: int = 0,
                 auto_reset: bool = True, want_final_obs: bool = False, config: CF2Config | None = None,
                 _spec=None, value_tables=None, copy_outputs: bool = False, **env_kwargs):
        if not torch.cuda.is_available():
            raise _native.CF2Error("BatchedCrazyflieEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.env_id = env_id
        self.spec = (_spec if _spec is not None else spec_for_id(env_id)) if config is None else None
        self.cfg = config if config is not None else build_config(
            self.spec, num_envs, seed=seed, env_id_offset=env_id_offset, auto_reset=auto_reset, **env_kwargs)
        self.num_envs = int(self.cfg.num_envs)
        self.obs_dim = obs_dim(self.cfg)
        self.lib = _native.load()
        self._ctx = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _native.check(self.lib.cf2_create(ctypes.byref(self.cfg), ctypes.byref(self._ctx)), "cf2_create")
        lay = _native.CF2Layout()
        _native.check(self.lib.cf2_layout_get(self._ctx, ctypes.byref(lay)), "cf2_layout_get")
        self.layout = lay
        n, d = self.num_envs, self.device
        self.obs = torch.zeros(n, self.obs_dim, dtype=torch.float32, device=d)
        self.rew = torch.zeros(n, dtype=torch.float32, device=d)
        self.done = torch.zeros(n, dtype=torch.uint8, device=d)
        self.trunc = torch.zeros(n, dtype=torch.uint8, device=d)
        self.cost = torch.zeros(n, dtype=torch.float32, device=d)
        self.level = torch.zeros(n, dtype=torch.float32, device=d)
        self._raw_ptrs = None                # step_raw's cached output addresses
        self.want_final_obs = want_final_obs
        self.last_collect_fused = False      # set by rollout.collect: its env-steps ran as cf2_collect_step
        self.final_obs = torch.zeros(n, self.obs_dim, dtype=torch.float32, device=d) if want_final_obs else None
        # the observations of the latest reset / step: self.obs, or the caller buffer (slab) that
        # step_into / rollout / step_raw wrote them to (what save_checkpoint saves)
        self._obs_latest = self.obs
        self._state_version = 0          # bumped by every call that changes the env state
        self._snap = None                # (version, state_f, state_i) of the last snapshot()
        self._tables = None
        # step() returns its output buffers themselves (overwritten by the next step) unless
        # copy_outputs, or step(copy=True)
        self.copy_outputs = bool(copy_outputs)
        # spaces (envs/base.py:139-148)
        self.observation_space = make_box(-1000.0, 1000.0, shape=(self.obs_dim,), dtype=np.float32)
        self.action_space = make_box(-1.0, 1.0, shape=(4,), dtype=np.float32)
        if value_tables is not None:
            self.bind_value_tables(value_tables)

    # ---- lifecycle ----
    def close(self):
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            torch.cuda.synchronize(self.device)
            self.lib.cf2_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    @property
    def stream(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    # ---- HJ tables (distur_gener.py:155 loads fastrack_{level}_15x15.npy each call; here once) ----
    def bind_hj_tables(self, V: torch.Tensor, table_of_level=None):
        """V: [T, 15,15,15,15,15,15] (or [T, 15**6]) float32 device tensor.  table_of_level maps the
        level index (0.0, 0.1, ..., 2.0; distur_gener.py:155 loads fastrack_{level}_15x15.npy per
        level) to a row of V.  Default: fixed-level envs use row 0; Boltzmann-level envs need one
        table per level (T == num_levels, identity map) or an explicit map."""
        V = V.reshape(V.shape[0], -1).contiguous().to(self.device, torch.float32)
        if V.shape[1] != 15 ** 6:
            raise ValueError("HJ value tables must be 15^6 grids")
        nl = int(self.cfg.num_levels)
        if table_of_level is None:
            if int(self.cfg.level_mode) == 1:   # Boltzmann level per episode
                if V.shape[0] != nl:
                    raise ValueError(f"this env draws one of {nl} levels per episode: bind {nl} tables (one per "
                                     f"level) or pass table_of_level explicitly")
                table_of_level = list(range(nl))
            else:
                table_of_level = [0] * nl
        if len(table_of_level) != nl:
            raise ValueError(f"table_of_level must have {nl} entries")
        t = (ctypes.c_int32 * int(self.cfg.num_levels))(*[int(x) for x in table_of_level])
        _native.check(self.lib.cf2_bind_hj_tables(self._ctx, V.data_ptr(), V.shape[0], t), "cf2_bind_hj_tables")
        self._tables = V   # keep alive

    def bind_value_tables(self, source):
        """Load and bind the HJ value tables this env reads (``load_value_tables``: the reference's
        ``fastrack_{level}_15x15.npy`` files from a directory, a dict by level, or an array)."""
        V, table_of_level = load_value_tables(source, self.cfg)
        self.bind_hj_tables(torch.from_numpy(V), table_of_level)

    # ---- gym-like API ----
    def reset(self, mask: torch.Tensor | None = None) -> torch.Tensor:
        m = None
        if mask is not None:
            m = mask.to(device=self.device, dtype=torch.uint8).contiguous()
            if self._obs_latest is None:
                # the rows of the envs that do not reset would keep stale values: the latest
                # observations went to a raw pointer (step_raw(obs_ptr=) or a raw collect step)
                raise ValueError("masked reset after a step into a raw obs pointer: the other envs' observations "
                                 "are not in env.obs; copy them into env.obs (or reset all envs) first")
        if mask is not None and self._obs_latest is not self.obs:
            # a masked reset writes only the reset envs' rows: the others must already be in self.obs
            self.obs.copy_(self._obs_latest)
        _native.check(self.lib.cf2_reset(self._ctx, _native.ptr(m), self.obs.data_ptr(), self.stream), "cf2_reset")
        self._state_version += 1
        self._obs_latest = self.obs
        return self.obs

    def step(self, actions: torch.Tensor, dstb: torch.Tensor | None = None, copy: bool | None = None):
        """One env-step of every env: (obs [N, D], rew [N], done [N] uint8, info).

        The returned tensors are this env's output buffers (self.obs, self.rew, ...), written
        again by the next step(): a caller that keeps a step's results across steps must clone
        them, or pass copy=True (or construct with copy_outputs=True) to get fresh tensors."""
        a = torch.as_tensor(actions)
        if a.device != self.device or a.dtype != torch.float32 or not a.is_contiguous() or a.data_ptr() % 16:
            a = a.to(device=self.device, dtype=torch.float32).contiguous()
            if a.data_ptr() % 16:
                a = a.clone()
        if a.shape != (self.num_envs, 4):
            raise ValueError(f"actions must be [{self.num_envs}, 4], got {tuple(a.shape)}")
        d = None
        if self.cfg.disturbance == DSTB_EXTERNAL:
            if dstb is None:
                raise ValueError("this env takes an external disturbance tensor dstb[N,3]")
            d = torch.as_tensor(dstb).to(device=self.device, dtype=torch.float32).contiguous()
            if d.shape != (self.num_envs, 3):
                raise ValueError(f"dstb must be [{self.num_envs}, 3], got {tuple(d.shape)}")
        if self.cfg.disturbance == DSTB_HJ and self._tables is None:
            raise _native.CF2Error("HJ-adversary env: bind value tables with bind_hj_tables() first")
        _native.check(self.lib.cf2_step(
            self._ctx, a.data_ptr(), _native.ptr(d), self.obs.data_ptr(), self.rew.data_ptr(), self.done.data_ptr(),
            self.trunc.data_ptr(), self.cost.data_ptr(), self.level.data_ptr(), _native.ptr(self.final_obs),
            self.stream), "cf2_step")
        self._state_version += 1
        self._obs_latest = self.obs
        info = {"cost": self.cost, "truncated": self.trunc, "disturbance_level": self.level}
        if self.final_obs is not None:
            info["final_obs"] = self.final_obs
        if self.copy_outputs if copy is None else copy:
            info = {k: v.clone() for k, v in info.items()}
            return self.obs.clone(), self.rew.clone(), self.done.clone(), info
        return self.obs, self.rew, self.done, info

    def step_into(self, actions: torch.Tensor, obs_out: torch.Tensor, rew_out: torch.Tensor, done_out: torch.Tensor,
                  trunc_out: torch.Tensor | None = None, cost_out: torch.Tensor | None = None,
                  final_obs_out: torch.Tensor | None = None):
        """step() writing straight into caller buffers (rollout storage); done/trunc are uint8.
        Every buffer is checked (device, dtype, shape, contiguity, alignment): the kernel trusts them."""
        n, od, dev = self.num_envs, self.obs_dim, self.device
        _check_buf(actions, "actions", (n, 4), torch.float32, dev, 16)
        _check_buf(obs_out, "obs_out", (n, od), torch.float32, dev, 16)
        _check_buf(rew_out, "rew_out", (n,), torch.float32, dev)
        _check_buf(done_out, "done_out", (n,), torch.uint8, dev, 1)
        _check_buf(trunc_out, "trunc_out", (n,), torch.uint8, dev, 1)
        _check_buf(cost_out, "cost_out", (n,), torch.float32, dev)
        _check_buf(final_obs_out, "final_obs_out", (n, od), torch.float32, dev, 8)
        if self.cfg.disturbance == DSTB_EXTERNAL:
            raise ValueError("this env takes an external disturbance tensor: use step(actions, dstb)")
        _native.check(self.lib.cf2_step(
            self._ctx, actions.data_ptr(), None, obs_out.data_ptr(), rew_out.data_ptr(), done_out.data_ptr(),
            _native.ptr(trunc_out), _native.ptr(cost_out), None, _native.ptr(final_obs_out), self.stream), "cf2_step")
        self._state_version += 1
        self._obs_latest = obs_out

    def collect_step_into(self, actions: torch.Tensor, obs_out: torch.Tensor, rew_out: torch.Tensor,
                          done_out: torch.Tensor, trunc_out: torch.Tensor | None, final_obs_out: torch.Tensor | None,
                          policy, act_out: torch.Tensor, val_out: torch.Tensor, logp_out: torch.Tensor) -> bool:
        """step_into() followed by policy.step_into(obs_out, act_out, val_out, logp_out) in one launch
        (cf2_collect_step: the collect loop's env.step + ac.step, algs/iwpg/iwpg.py:377-380).  The
        outputs are bit-identical to the two calls.  Returns False, having launched nothing, where
        no fused instance is built (cf2sim.h); the caller then makes the two calls."""
        n, od, dev = self.num_envs, self.obs_dim, self.device
        _check_buf(actions, "actions", (n, 4), torch.float32, dev, 16)
        _check_buf(obs_out, "obs_out", (n, od), torch.float32, dev, 16)
        _check_buf(rew_out, "rew_out", (n,), torch.float32, dev)
        _check_buf(done_out, "done_out", (n,), torch.uint8, dev, 1)
        _check_buf(trunc_out, "trunc_out", (n,), torch.uint8, dev, 1)
        _check_buf(final_obs_out, "final_obs_out", (n, od), torch.float32, dev, 8)
        _check_buf(act_out, "act_out", (n, 4), torch.float32, dev, 16)
        _check_buf(val_out, "val_out", (n,), torch.float32, dev)
        _check_buf(logp_out, "logp_out", (n,), torch.float32, dev)
        if self.cfg.disturbance == DSTB_EXTERNAL:
            raise ValueError("this env takes an external disturbance tensor: use step(actions, dstb)")
        if policy.obs_dim != od:
            raise ValueError(f"policy obs_dim {policy.obs_dim} != env obs_dim {od}")
        st = self.lib.cf2_collect_step(
            self._ctx, actions.data_ptr(), obs_out.data_ptr(), rew_out.data_ptr(), done_out.data_ptr(),
            _native.ptr(trunc_out), _native.ptr(final_obs_out), policy.w.data_ptr(), od, policy.prec, policy.seed,
            policy.counter & 0xFFFFFFFF, int(self.cfg.env_id_offset), act_out.data_ptr(), val_out.data_ptr(),
            logp_out.data_ptr(), self.stream)
        if st == _native.CF2_ERR_UNSUPPORTED:
            return False
        _native.check(st, "cf2_collect_step")
        policy.counter += 1
        self._state_version += 1
        self._obs_latest = obs_out
        return True

    def collect_step_raw(self, act: int, obs: int, rew: int, done: int, trunc: int, final_obs: int, policy,
                         act_out: int, val_out: int, logp_out: int) -> bool:
        """collect_step_into on raw device pointers (rollout.collect's loop after its first step,
        whose slabs collect_step_into has checked; the C ABI still rejects null or misaligned
        pointers): keeps the host's per-step cost well under the kernel's."""
        st = self.lib.cf2_collect_step(self._ctx, act, obs, rew, done, trunc, final_obs, policy.w_ptr, self.obs_dim,
                                       policy.prec, policy.seed, policy.counter & 0xFFFFFFFF, int(self.cfg.env_id_offset),
                                       act_out, val_out, logp_out, self.stream)
        if st == _native.CF2_ERR_UNSUPPORTED:
            return False
        _native.check(st, "cf2_collect_step")
        policy.counter += 1
        self._state_version += 1
        self._obs_latest = None          # rollout.collect points it at the slab afterwards
        return True

    def collect_rollout_into(self, act: torch.Tensor, obs_out: torch.Tensor, rew_out: torch.Tensor,
                             done_out: torch.Tensor, trunc_out: torch.Tensor | None, final_obs_out: torch.Tensor | None,
                             policy, val_out: torch.Tensor, logp_out: torch.Tensor) -> bool:
        """K steps of the collect loop in one launch (cf2_collect_rollout): K = obs_out.shape[0].
        act [K+1, N, 4]: slab 0 holds the first step's actions, slabs 1..K receive the policy's
        samples on the observations after steps 0..K-1, with val_out / logp_out [K+1, N] (slab 0
        untouched); obs_out [K, N, D] (slab k = the observation after step k), rew / done / trunc
        [K, N], final_obs [K, N, D].  Bit-identical to K collect_step_into calls.  Returns False,
        having launched nothing, where no fused instance is built."""
        K = int(obs_out.shape[0])
        n, od, dev = self.num_envs, self.obs_dim, self.device
        _check_buf(act, "act", (K + 1, n, 4), torch.float32, dev, 16)
        _check_buf(obs_out, "obs_out", (K, n, od), torch.float32, dev, 8)
        _check_buf(rew_out, "rew_out", (K, n), torch.float32, dev)
        _check_buf(done_out, "done_out", (K, n), torch.uint8, dev, 1)
        _check_buf(trunc_out, "trunc_out", (K, n), torch.uint8, dev, 1)
        _check_buf(final_obs_out, "final_obs_out", (K, n, od), torch.float32, dev, 8)
        _check_buf(val_out, "val_out", (K + 1, n), torch.float32, dev)
        _check_buf(logp_out, "logp_out", (K + 1, n), torch.float32, dev)
        if self.cfg.disturbance == DSTB_EXTERNAL:
            raise ValueError("this env takes an external disturbance tensor: use step(actions, dstb)")
        if policy.obs_dim != od:
            raise ValueError(f"policy obs_dim {policy.obs_dim} != env obs_dim {od}")
        st = self.lib.cf2_collect_rollout(
            self._ctx, K, act.data_ptr(), obs_out.data_ptr(), rew_out.data_ptr(), done_out.data_ptr(),
            _native.ptr(trunc_out), _native.ptr(final_obs_out), policy.w.data_ptr(), od, policy.prec, policy.seed,
            policy.counter & 0xFFFFFFFF, int(self.cfg.env_id_offset), val_out.data_ptr(), logp_out.data_ptr(),
            self.stream)
        if st == _native.CF2_ERR_UNSUPPORTED:
            return False
        _native.check(st, "cf2_collect_rollout")
        policy.counter += K
        self._state_version += 1
        self._obs_latest = obs_out[K - 1]
        return True

    def rollout(self, actions: torch.Tensor, obs_out: torch.Tensor | None = None, rew_out=None, done_out=None,
                trunc_out=None, cost_out=None, level_out=None, final_obs_out=None):
        """K env-steps in one fused launch (cf2_rollout): actions [K, N, 4]; returns (obs [K, N, D],
        rew [K, N], done [K, N], info with truncated / cost / disturbance_level [K, N] and
        final_obs [K, N, D] when the env keeps final observations).  Identical to K step() calls
        with the same actions; the state stays in registers across the K steps."""
        K = int(actions.shape[0])
        n, od, dev = self.num_envs, self.obs_dim, self.device
        _check_buf(actions, "actions", (K, n, 4), torch.float32, dev, 16)
        obs_out = obs_out if obs_out is not None else torch.empty(K, n, od, device=dev)
        rew_out = rew_out if rew_out is not None else torch.empty(K, n, device=dev)
        done_out = done_out if done_out is not None else torch.empty(K, n, dtype=torch.uint8, device=dev)
        trunc_out = trunc_out if trunc_out is not None else torch.empty(K, n, dtype=torch.uint8, device=dev)
        cost_out = cost_out if cost_out is not None else torch.empty(K, n, device=dev)
        level_out = level_out if level_out is not None else torch.empty(K, n, device=dev)
        if final_obs_out is None and self.want_final_obs:
            final_obs_out = torch.empty(K, n, od, device=dev)
        _check_buf(obs_out, "obs_out", (K, n, od), torch.float32, dev, 8)
        _check_buf(rew_out, "rew_out", (K, n), torch.float32, dev)
        _check_buf(done_out, "done_out", (K, n), torch.uint8, dev, 1)
        _check_buf(trunc_out, "trunc_out", (K, n), torch.uint8, dev, 1)
        _check_buf(cost_out, "cost_out", (K, n), torch.float32, dev)
        _check_buf(level_out, "level_out", (K, n), torch.float32, dev)
        _check_buf(final_obs_out, "final_obs_out", (K, n, od), torch.float32, dev, 8)
        if self.cfg.disturbance == DSTB_HJ and self._tables is None:
            raise _native.CF2Error("HJ-adversary env: bind value tables with bind_hj_tables() first")
        _native.check(self.lib.cf2_rollout(
            self._ctx, K, actions.data_ptr(), n * 4, obs_out.data_ptr(), rew_out.data_ptr(), done_out.data_ptr(),
            trunc_out.data_ptr(), cost_out.data_ptr(), level_out.data_ptr(), _native.ptr(final_obs_out), self.stream),
            "cf2_rollout")
        self._state_version += 1
        self._obs_latest = obs_out[K - 1]
        info = {"cost": cost_out, "truncated": trunc_out, "disturbance_level": level_out}
        if final_obs_out is not None:
            info["final_obs"] = final_obs_out
        return obs_out, rew_out, done_out, info

    def step_raw(self, act_ptr: int, obs_ptr: int | None = None, full_info: bool = True, done_ptr: int | None = None):
        """Launch one env-step with a raw device pointer to [N, 4] float32 actions (benchmark /
        graph-capture helper; the pointer is not checked).  full_info: also write the truncation,
        cost and level outputs step() returns in info (the reference's compute_info runs every step,
        envs/hover_free.py:138-166).  With obs_ptr the observations go to that raw buffer, which
        save_checkpoint cannot see: pass it the observations explicitly.  done_ptr: the uint8 done
        flags go to that buffer instead of self.done (the delta obs exchange packs them later)."""
        self._obs_latest = self.obs if obs_ptr is None else None
        self._state_version += 1
        p = self._raw_ptrs
        if p is None:          # the output buffers are allocated once: their addresses are cached
            p = self._raw_ptrs = (self.obs.data_ptr(), self.rew.data_ptr(), self.done.data_ptr(), self.trunc.data_ptr(),
                                  self.cost.data_ptr(), self.level.data_ptr())
        st = self.lib.cf2_step(self._ctx, act_ptr, None, obs_ptr or p[0], p[1], done_ptr or p[2],
                               p[3] if full_info else None, p[4] if full_info else None, p[5] if full_info else None,
                               None, torch.cuda.current_stream(self.device).cuda_stream)
        if st != 0:
            _native.check(st, "cf2_step")

    def _raw_step_outputs(self):
        """For an env-step launched outside step_raw (the native exchange's cf2_xchg_env_step, whose
        observations go to the exchange's buffers): the reward / truncation / cost / level output
        addresses; the step is recorded as step_raw records one."""
        self._obs_latest = None
        self._state_version += 1
        p = self._raw_ptrs
        if p is None:
            p = self._raw_ptrs = (self.obs.data_ptr(), self.rew.data_ptr(), self.done.data_ptr(), self.trunc.data_ptr(),
                                  self.cost.data_ptr(), self.level.data_ptr())
        return p[1], p[3], p[4], p[5]

    # ---- state snapshot ----
    def get_state(self):
        sf = torch.empty(self.layout.num_float_fields, self.num_envs, dtype=torch.float32, device=self.device)
        si = torch.empty(self.layout.num_int_fields, self.num_envs, dtype=torch.int32, device=self.device)
        _native.check(self.lib.cf2_get_state(self._ctx, sf.data_ptr(), si.data_ptr(), self.stream), "cf2_get_state")
        return sf, si

    def set_state(self, sf: torch.Tensor, si: torch.Tensor):
        sf = sf.to(self.device, torch.float32).contiguous()
        si = si.to(self.device, torch.int32).contiguous()
        if sf.shape != (self.layout.num_float_fields, self.num_envs) or si.shape != (self.layout.num_int_fields, self.num_envs):
            raise ValueError("state tensors do not match cf2_layout")
        _native.check(self.lib.cf2_set_state(self._ctx, sf.data_ptr(), si.data_ptr(), self.stream), "cf2_set_state")
        self._state_version += 1

    def check_device_errors(self, clear: bool = True):
        """Raise CF2Error if a kernel of this batch recorded a device-side error (cf2_device_errors:
        a helper wave that gave up waiting for an LDS hand-over).  Synchronises the device."""
        flags = ctypes.c_uint32(0)
        _native.check(self.lib.cf2_device_errors(self._ctx, ctypes.byref(flags), int(clear)), "cf2_device_errors")
        if flags.value:
            raise _native.CF2Error(f"device error flags 0x{flags.value:x} (1: a helper wave's LDS hand-over timed out)")

    def invalidate(self):
        """Mark the cached snapshot (and the observations' owner) stale.  Needed after anything
        that changes the state without going through this object: replaying a hipGraph that
        captured step_raw / step_into, or calling the C ABI on self._ctx directly."""
        self._state_version += 1

    def snapshot(self):
        """get_state(), cached until the next call that changes the state (step, reset, rollout,
        set_state, a physics-plugin step): repeated reads of agent attributes between two steps
        cost one conversion kernel, not one each.  The tensors are shared: do not modify them.
        A graph replay or a direct C-ABI call does not update the cache: call invalidate()."""
        if self._snap is None or self._snap[0] != self._state_version:
            sf, si = self.get_state()
            self._snap = (self._state_version, sf, si)
        return self._snap[1], self._snap[2]

    # ---- checkpoint / resume (the reference never checkpoints env state) ----
    def save_checkpoint(self, path: str, obs: torch.Tensor | None = None):
        """Write the whole batch to a safetensors file: the state snapshot, the current
        observations and the raw cf2_config (seed, offsets and every constant), so that
        ``from_checkpoint`` resumes bit-identically (every draw is keyed by the seed, the global
        env id and the per-env counter in the snapshot).  Bound HJ tables are not saved.

        The observations saved are those of the latest reset / step / step_into / rollout call
        (for step_into and rollout: the caller's buffer, read now, so it must still hold them), or
        ``obs`` if given ([N, obs_dim]; required after step_raw with a raw obs pointer)."""
        from safetensors.torch import save_file
        cur = obs if obs is not None else self._obs_latest
        if cur is None:
            raise ValueError("the latest observations went to a raw buffer (step_raw obs_ptr): pass obs=")
        if tuple(cur.shape) != (self.num_envs, self.obs_dim):
            raise ValueError(f"obs must be [{self.num_envs}, {self.obs_dim}]")
        sf, si = self.get_state()
        torch.cuda.synchronize(self.device)
        cfg = torch.frombuffer(bytearray(bytes(self.cfg)), dtype=torch.uint8)
        save_file({"state_f": sf.cpu(), "state_i": si.cpu(), "obs": cur.detach().float().cpu().contiguous(),
                   "config": cfg}, path,
                  metadata={"env_id": self.env_id, "abi_version": str(self.lib.cf2_abi_version()),
                            "want_final_obs": str(int(self.want_final_obs))})

    def load_checkpoint(self, path: str):
        """Restore a batch saved by ``save_checkpoint`` into this env, whose configuration must be
        the saved one (ValueError otherwise)."""
        from safetensors import safe_open
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
            t = {k: f.get_tensor(k) for k in f.keys()}
        if meta.get("abi_version") != str(self.lib.cf2_abi_version()):
            raise ValueError(f"checkpoint written by ABI {meta.get('abi_version')}, library is "
                             f"{self.lib.cf2_abi_version()}")
        if bytes(t["config"].numpy().tobytes()) != bytes(self.cfg):
            raise ValueError("checkpoint configuration differs from this env's")
        self.set_state(t["state_f"], t["state_i"])
        self.obs.copy_(t["obs"].to(self.device))
        self._obs_latest = self.obs

    @classmethod
    def from_checkpoint(cls, path: str, device=None) -> "BatchedCrazyflieEnv":
        """A new env holding the batch saved by ``save_checkpoint`` (same config, state, obs)."""
        from safetensors import safe_open
        with safe_open(path, framework="pt") as f:
            meta = f.metadata() or {}
            raw = f.get_tensor("config").numpy().tobytes()
        if len(raw) != ctypes.sizeof(CF2Config):
            raise ValueError("checkpoint config size does not match this build's cf2_config")
        cfg = CF2Config.from_buffer_copy(raw)
        env = cls(meta.get("env_id", ""), int(cfg.num_envs), device=device, config=cfg,
                  want_final_obs=meta.get("want_final_obs") == "1")
        env.load_checkpoint(path)
        return env

    def gather_observations(self, group=None, out: torch.Tensor | None = None) -> torch.Tensor:
        """RCCL all-gather of every rank's obs slab (optional policy-side exchange; the physics
        itself needs no collective).  Returns [sum of N over ranks, obs_dim] in rank order: a fresh
        tensor per call, or ``out`` when given (opt-in buffer reuse: the next call with the same
        ``out`` overwrites it).  The observations gathered are the latest step's or reset's."""
        from .dist import exchange_sizes, gather_rows
        key = id(group)
        if getattr(self, "_gather_key", None) != key:   # shard sizes: exchanged once per group
            self._gather_sizes = exchange_sizes(self.num_envs, group)
            self._gather_key = key
        src = self._obs_latest if self._obs_latest is not None else self.obs
        if out is not None:
            _check_buf(out, "out", (sum(self._gather_sizes), self.obs_dim), torch.float32, self.device)
        return gather_rows(src, group, sizes=self._gather_sizes, out=out)


def hj_disturbance(V: torch.Tensor, states: torch.Tensor, level: float, cfg: CF2Config | None = None):
    """Batched ``distur_gener(states, level)`` (distur_gener.py:19-183) on the GPU:
    states [n, 6] = [roll, pitch, yaw, p, q, r] -> (u_opt [n,3], d_opt [n,3])."""
    lib = _native.load()
    if cfg is None:
        cfg = build_config("DroneHoverBulletFreeEnvWithAdversary-v0", 1)
    if not float(level) <= 3.0:
        raise AssertionError("disturbance level must be <= 3.0 (distur_gener.py:154)")
    s = states.to(torch.float32).contiguous()
    n = s.shape[0]
    d = torch.empty(n, 3, dtype=torch.float32, device=s.device)
    u = torch.empty(n, 3, dtype=torch.float32, device=s.device)
    Vf = V.reshape(-1).to(s.device, torch.float32).contiguous()
    _native.check(lib.cf2_hj_disturbance(ctypes.byref(cfg), Vf.data_ptr(), s.data_ptr(), n, float(level),
                                         d.data_ptr(), u.data_ptr(), torch.cuda.current_stream(s.device).cuda_stream),
                  "cf2_hj_disturbance")
    return u, d
