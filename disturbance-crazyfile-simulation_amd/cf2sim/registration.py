"""Single-env gym-style adapter over the batched HIP env, with the reference's env ids.

The reference registers its hover envs with gym (phoenix_drone_simulation/__init__.py:8-109,
``max_episode_steps=500``) and callers do ``env = gym.make(id); obs = env.reset();
obs, r, done, info = env.step(a)`` (tests/test_envs.py:96-123, algs/iwpg/iwpg.py:372-410).
``make(id)`` returns an object with that API, backed by a 1-env ``BatchedCrazyflieEnv``:

* ``reset() -> np.ndarray[obs_dim]`` float64 (the reference builds obs with numpy float64 ops)
* ``step(a) -> (obs, float r, bool done, dict info)``, ``info`` = compute_info() keys
  (``cost``, ``disturbance_level``, and ``xyz_limit`` / ``rpy`` / ``xzy_dot`` / ``rpy_dot`` for the
  constraints the step violates, envs/hover_free.py:138-166) plus ``TimeLimit.truncated`` when gym's
  TimeLimit(500) ends the episode (gym 0.19 TimeLimit semantics: done = terminal or truncated; no
  auto-reset)
* HJ-adversary ids read value tables: ``make(id, value_tables=dir)`` loads the reference's
  ``fastrack_{level}_15x15.npy`` files (distur_gener.py:155; a directory, a dict by level or an
  array, see vec_env.load_value_tables); ``env.bind_hj_tables(...)`` rebinds them
* ``observation_space`` Box(-1000, 1000, (34,), float32) / (42,) without noise, ``action_space``
  Box(-1, 1, (4,), float32) (envs/base.py:139-148); ``metadata`` as envs/base.py:24
* ``seed(s)`` re-seeds the Philox stream (the reference re-seeds numpy's global RNG)

The physics plugin is chosen by name like the reference's ``physics=`` string
(envs/base.py:223-231): 'PybulletPhysicsWithAdversary', 'PyBulletPhysics' (the Bullet
restatement), 'SimplePhysics' (physics.py:127-200) and 'HipBatchedPhysics' (whatever the env id
uses).  Unknown names fail like the reference's assert.  The same names are classes with the
reference's plugin contract in cf2sim.physics.
"""
from __future__ import annotations

import numpy as np

from .config import ENV_SPECS, PHYS_BULLET, PHYS_SIMPLE, REFERENCE_IDS, spec_for_id  # noqa: F401

PHYSICS_PLUGINS = {
    "PybulletPhysicsWithAdversary": PHYS_BULLET,   # envs/physics.py:202
    "PyBulletPhysics": PHYS_BULLET,                # envs/physics.py:79
    "SimplePhysics": PHYS_SIMPLE,                  # envs/physics.py:127
    "HipBatchedPhysics": None,                     # the env id's own physics, fused HIP kernel
}


def resolve_physics(physics: str | None, default: int) -> int:
    """The physics type an env runs for the reference's ``physics=`` string; unknown names fail
    like the reference's assert (envs/base.py:224-225).  The plugin classes themselves
    (constructor, set_parameters, step_forward) are in cf2sim.physics."""
    if physics is None:
        return default
    if physics not in PHYSICS_PLUGINS:
        raise AssertionError(f"Physics={physics} not found.")
    p = PHYSICS_PLUGINS[physics]
    return default if p is None else p


# registered ids + the framework's extension ids (C2 const wind, C4 gust) of BASELINE.json
registry = {s.registered_id: s for s in ENV_SPECS.values() if s.registered_id}


class CrazyflieEnv:
    metadata = {"render.modes": ["human", "rgb_array"]}   # envs/base.py:24
    reward_range = (-float("inf"), float("inf"))

    def __init__(self, env_id: str, seed: int = 0, device=None, physics: str | None = None, value_tables=None,
                 **env_kwargs):
        from .vec_env import BatchedCrazyflieEnv
        self.spec = spec_for_id(env_id)
        self._value_tables = value_tables
        self.env_id = env_id
        self._kwargs = dict(env_kwargs)
        self._device = device
        self._physics = resolve_physics(physics, self.spec.physics)
        self.max_episode_steps = int(self._kwargs.pop("max_episode_steps", 500))
        self._cls = BatchedCrazyflieEnv
        self._seed = int(seed)
        self._make()

    def _make(self):
        from dataclasses import replace
        spec = replace(self.spec, physics=self._physics)
        # TimeLimit is applied here (as gym's wrapper does), the kernel only sees terminal states
        self._env = self._cls(spec.registered_id or self.env_id, 1, seed=self._seed, device=self._device,
                              auto_reset=False, max_episode_steps=0, _spec=spec, **self._kwargs)
        self.observation_space = self._env.observation_space
        self.action_space = self._env.action_space
        if self._value_tables is not None:
            self._env.bind_value_tables(self._value_tables)
        self._t = 0
        self._needs_reset = True
        self._last_action = np.zeros(4, np.float32)
        self._field_idx = None
        # penalty terms of the last compute_reward (envs/hover_free.py:61-66, 227-232), read by the
        # reference's learner for logging (algs/iwpg/iwpg.py:531-532)
        self.penalty_log = self.penalty_rpy_log = self.penalty_crash_log = 0.0
        self.penalty_z_log = self.penalty_rpy_dot_log = self.penalty_velocity_log = 0.0

    def bind_hj_tables(self, value_tables, table_of_level=None):
        """Bind the HJ value tables of an adversary env: a directory with the reference's
        ``fastrack_{level}_15x15.npy`` files (or the reference's repository root), a dict
        {level: table}, or an array of tables (``table_of_level`` maps each level to a row).  Kept
        across ``seed()``."""
        import torch
        if table_of_level is not None:
            self._env.bind_hj_tables(torch.as_tensor(value_tables), table_of_level)
        else:
            self._env.bind_value_tables(value_tables)
        self._value_tables = value_tables if table_of_level is None else None
        if table_of_level is not None:
            self._tables_explicit = (value_tables, table_of_level)

    @property
    def disturbance_level(self) -> float:        # read by iwpg.py:408
        return float(self._env.level[0].item())

    def seed(self, seed=None):
        self._seed = int(seed) if seed is not None else 0
        self._env.close()
        self._make()
        if getattr(self, "_tables_explicit", None) is not None and self._value_tables is None:
            import torch
            self._env.bind_hj_tables(torch.as_tensor(self._tables_explicit[0]), self._tables_explicit[1])
        return [self._seed]

    def _state_fields(self):
        """Indices into the state snapshot of what the host side reads per step: pos, quat, vel,
        omega, rpy (Simple physics) and the action buffer's last row (drone.last_action)."""
        if getattr(self, "_field_idx", None) is None:
            import torch
            L = self._env.layout
            last = L.f_abuf + 4 * (int(self._env.cfg.buf_size) - 1)
            idx = ([L.f_pos + k for k in range(3)] + [L.f_quat + k for k in range(4)] + [L.f_vel + k for k in range(3)]
                   + [L.f_omega + k for k in range(3)] + [L.f_rpy + k for k in range(3)] + [last + k for k in range(4)])
            self._field_idx = torch.tensor(idx, dtype=torch.long, device=self._env.device)
        return self._field_idx

    def reset(self) -> np.ndarray:
        import torch
        obs = self._env.reset()
        self._t = 0
        self._needs_reset = False
        sf, _ = self._env.snapshot()
        # one device -> host transfer: the observation row and the action buffer's last row
        h = torch.cat([obs[0], sf[self._state_fields(), 0]]).cpu().double().numpy()
        od = self._env.obs_dim
        self._last_action = h[od + 16:od + 20].astype(np.float32)
        return h[:od]

    def step(self, action):
        import torch
        if self._needs_reset:
            raise RuntimeError("call reset() before step() (gym TimeLimit semantics)")
        act = np.asarray(action, dtype=np.float32).reshape(4)
        a = torch.as_tensor(act.reshape(1, 4), device=self._env.device)
        obs, rew, done, info = self._env.step(a)
        sf, _ = self._env.snapshot()
        # everything the host needs from this step in ONE device -> host transfer (one stream
        # sync): obs row, reward, done, cost, level and the state fields the penalty log reads
        h = torch.cat([obs[0], rew, done.float(), info["cost"], info["disturbance_level"],
                       sf[self._state_fields(), 0]]).cpu().double().numpy()
        od = self._env.obs_dim
        r, terminal, cost, level = float(h[od]), bool(h[od + 1] != 0), float(h[od + 2]), float(h[od + 3])
        self._t += 1
        rpy, rpy_dot = self._log_penalties(act, terminal, h[od + 4:])
        info_out = self._constraint_info(h[od + 4:], rpy, act)
        info_out.update({"cost": cost, "disturbance_level": level})
        truncated = self._t >= self.max_episode_steps > 0
        if truncated and not terminal:
            info_out["TimeLimit.truncated"] = True
        d = terminal or truncated
        if d:
            self._needs_reset = True
        return h[:od], r, d, info_out

    def _log_penalties(self, action, terminal: bool, st):
        """The individual terms of compute_reward (hover_free.py:206-235) from the env's state after
        the step (host-side, single-env adapter only; the batched kernel computes the reward).
        st: pos, quat, vel, omega, rpy, last action (_state_fields order), float64."""
        c = self._env.cfg
        p, q, v, w = st[0:3], st[3:7], st[7:10], st[10:13]
        if int(c.physics) == PHYS_SIMPLE:
            rpy, rpy_dot = st[13:16], w
        else:
            x, y, z, qw = q
            sarg = min(max(-2.0 * (x * z - qw * y), -1.0), 1.0)
            rpy = np.array([np.arctan2(2 * (y * z + qw * x), qw * qw - x * x - y * y + z * z), np.arcsin(sarg),
                            np.arctan2(2 * (x * y + qw * z), qw * qw + x * x - y * y - z * z)])
            s2 = 2.0 / float(q @ q)
            R = np.array([[1 - s2 * (y * y + z * z), s2 * (x * y - qw * z), s2 * (x * z + qw * y)],
                          [s2 * (x * y + qw * z), 1 - s2 * (x * x + z * z), s2 * (y * z - qw * x)],
                          [s2 * (x * z - qw * y), s2 * (y * z + qw * x), 1 - s2 * (x * x + y * y)]])
            rpy_dot = R.T @ w
        tgt_rpy, tgt_rate, tgt_pos = np.array(c.target_rpy[:]), np.array(c.target_rate[:]), np.array(c.target_pos[:])
        pen_action = c.penalty_action * np.linalg.norm(0.5 * (np.clip(action, -1, 1) + 1))
        pen_arp = c.penalty_arp * np.linalg.norm(action - self._last_action)
        self.penalty_rpy_log = c.penalty_angle * np.linalg.norm(rpy - tgt_rpy)
        self.penalty_rpy_dot_log = c.penalty_spin * np.linalg.norm(rpy_dot - tgt_rate)
        self.penalty_crash_log = c.penalty_terminal if terminal else 0.0
        self.penalty_velocity_log = c.penalty_velocity * np.linalg.norm(v)
        self.penalty_log = (self.penalty_rpy_log + pen_arp + self.penalty_rpy_dot_log + self.penalty_velocity_log
                            + pen_action + self.penalty_crash_log)
        self.penalty_z_log = c.penalty_z * abs(p[2] - tgt_pos[2])
        self._last_action = action
        return rpy, rpy_dot

    def _constraint_info(self, st, rpy, action) -> dict:
        """The conditional keys of compute_info (envs/hover_free.py:138-166, envs/hover.py:116-144)
        from the state after the step.  state = get_state() = [xyz, quat, xyz_dot, rpy_dot (body),
        last_action] (agents.py:339-348), and the reference indexes state[10:13] (the body rates)
        as 'xzy_dot' and state[13:16] (the first three last-action entries) as 'rpy_dot': reproduced
        as written.  last_action is the action just applied (apply_action, agents.py:263).  The
        kernel's cost flag (info['cost']) uses the same conditions."""
        c = self._env.cfg
        p, q, v, w = st[0:3], st[3:7], st[7:10], st[10:13]
        la = np.asarray(action, dtype=np.float64)
        if int(c.physics) == PHYS_SIMPLE:
            wb = w
        else:
            x, y, z, qw = q
            s2 = 2.0 / float(q @ q)
            R = np.array([[1 - s2 * (y * y + z * z), s2 * (x * y - qw * z), s2 * (x * z + qw * y)],
                          [s2 * (x * y + qw * z), 1 - s2 * (x * x + z * z), s2 * (y * z - qw * x)],
                          [s2 * (x * z - qw * y), s2 * (y * z + qw * x), 1 - s2 * (x * x + y * y)]])
            wb = R.T @ w
        state = np.concatenate([p, q, v, wb, la])
        info = {}
        if abs(p[0]) > c.cost_xy_lim or abs(p[1]) > c.cost_xy_lim or p[2] > c.cost_z_lim:
            info["xyz_limit"] = state[:3]
        if (np.abs(np.asarray(rpy)[:2]) > c.cost_rp_lim).any():
            info["rpy"] = np.asarray(rpy)
        if (np.abs(state[10:13]) > c.cost_vel_lim).any():
            info["xzy_dot"] = state[10:13]
        if (np.abs(state[13:16]) > c.cost_rate_lim).any():
            info["rpy_dot"] = state[13:16] * 180 / np.pi
        return info

    def render(self, mode="human"):
        raise NotImplementedError("rendering is outside the accelerated path (DESIGN.md 'Out of scope')")

    def close(self):
        self._env.close()


def make(env_id: str, **kwargs) -> CrazyflieEnv:
    """``gym.make(env_id)`` equivalent for the hover ids (REFERENCE_IDS) and the extension ids."""
    spec_for_id(env_id)   # raises KeyError / NotImplementedError for unknown / out-of-scope ids
    return CrazyflieEnv(env_id, **kwargs)


__all__ = ["make", "registry", "CrazyflieEnv", "resolve_physics", "PHYSICS_PLUGINS", "REFERENCE_IDS"]
