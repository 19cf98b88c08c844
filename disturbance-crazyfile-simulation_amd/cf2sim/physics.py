"""Physics plugins with the reference's physics-class contract, run by the HIP physics kernel.

The reference picks its physics by name and builds it around the env's drone and bullet client
(phoenix_drone_simulation/envs/base.py:223-232)::

    physics_cls = getattr(phoenix_physics, physics)            # e.g. 'PybulletPhysicsWithAdversary'
    self.physics = physics_cls(self.drone, self.bc, time_step=self.time_step)
    self.physics.set_parameters(time_step=..., number_solver_iterations=...)   # base.py:264 (DR)
    self.physics.step_forward(action, dstb)                                     # hover_free.py:431

``import cf2sim.physics as phoenix_physics`` makes the same lines work here.  The classes keep
the reference's names, constructor ``(drone, bc, time_step, gravity=9.81,
number_solver_iterations=5, use_ground_effect=False)`` (envs/physics.py:8-25),
``set_parameters(time_step, number_solver_iterations)`` (:60-68, :81-89, :203-211) and
``step_forward(action[, dstb])`` (:91-124, :130-200, :213-250).  What differs is batching: the
``drone`` is a :class:`BatchedDrone` of N agents whose state stays in HBM, ``action`` is an
[N, 4] device tensor, and one ``step_forward`` advances all N drones by one physics sub-step in
one launch of ``cf2_physics_step`` (include/cf2sim.h).  ``bc`` (the PyBullet client) has no role
since the rigid-body step is the kernel's own; any value is accepted and kept.

There is no CPU fallback: every class needs libcf2sim.so and a GPU.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native
from .config import PHYS_BULLET, PHYS_SIMPLE
from .registration import PHYSICS_PLUGINS, resolve_physics  # noqa: F401  (re-exported)

__all__ = ["BatchedDrone", "BasePhysics", "PyBulletPhysics", "PybulletPhysicsWithAdversary", "SimplePhysics",
           "HipBatchedPhysics", "PHYSICS_PLUGINS", "resolve_physics"]

# drone model -> the env id whose agent it is (envs/base.py:209-214 builds the agent by model name)
_DRONE_MODEL_ENV = {
    "cf21x_bullet": "DroneHoverBulletFreeEnvWithoutAdversary-v0",
    "cf21x_sys_eq": "DroneHoverSimpleEnv-v0",
}


class BatchedDrone:
    """N CrazyFlie agents in one cf2 context: the object a physics plugin acts on.

    Mirrors the attributes of the reference's agents that the physics reads and writes
    (envs/agents.py: ``xyz``, ``quaternion``, ``xyz_dot``, ``rpy``, ``rpy_dot``, ``x``), as [N, k]
    float32 device tensors read from the state snapshot.  ``reset()`` is the env's reset of the
    agents (DroneBaseEnv.reset envs/base.py:420-464 incl. task reset and domain randomisation)."""

    def __init__(self, drone_model: str = "cf21x_bullet", num_drones: int = 1, seed: int = 0, device=None,
                 env_id: str | None = None, config=None, **env_kwargs):
        """config: a full cf2sim.config.CF2Config (num_envs = the number of drones) instead of the
        env id's defaults plus env_kwargs."""
        from .vec_env import BatchedCrazyflieEnv
        if config is not None:
            self.env = BatchedCrazyflieEnv(env_id or "", int(config.num_envs), device=device, config=config)
            self.drone_model = "cf21x_bullet" if self.physics_type == PHYS_BULLET else "cf21x_sys_eq"
            self.num_drones = self.env.num_envs
            return
        if env_id is None:
            if drone_model not in _DRONE_MODEL_ENV:
                raise NotImplementedError(f"drone_model={drone_model}")   # envs/base.py:214
            env_id = _DRONE_MODEL_ENV[drone_model]
        env_kwargs.setdefault("max_episode_steps", 0)
        self.env = BatchedCrazyflieEnv(env_id, num_drones, seed=seed, device=device, auto_reset=False, **env_kwargs)
        self.drone_model = "cf21x_bullet" if self.physics_type == PHYS_BULLET else "cf21x_sys_eq"
        self.num_drones = self.env.num_envs

    @property
    def physics_type(self) -> int:
        return int(self.env.cfg.physics)

    @property
    def device(self):
        return self.env.device

    def reset(self, mask: torch.Tensor | None = None) -> torch.Tensor:
        return self.env.reset(mask)

    def _fields(self):
        sf, _ = self.env.snapshot()          # one conversion per state change, shared by the properties
        return sf, self.env.layout           # (each property returns its own copy: .clone())

    @property
    def xyz(self):
        sf, L = self._fields()
        return sf[L.f_pos:L.f_pos + 3].T.clone(memory_format=torch.contiguous_format)

    @property
    def quaternion(self):
        sf, L = self._fields()
        return sf[L.f_quat:L.f_quat + 4].T.clone(memory_format=torch.contiguous_format)

    @property
    def xyz_dot(self):
        sf, L = self._fields()
        return sf[L.f_vel:L.f_vel + 3].T.clone(memory_format=torch.contiguous_format)

    @property
    def x(self):
        """First-order motor state (agents.py:288), hi + lo words of the compensated pair."""
        sf, L = self._fields()
        return (sf[L.f_motor:L.f_motor + 4].double() + sf[L.f_motor_lo:L.f_motor_lo + 4].double()).T.float()

    @property
    def rpy_dot(self):
        """Body angular rates (update_information agents.py:434-453: R(q)^T omega_world)."""
        sf, L = self._fields()
        w = sf[L.f_omega:L.f_omega + 3].T
        if self.physics_type == PHYS_SIMPLE:
            return w.clone(memory_format=torch.contiguous_format)
        return torch.einsum("nji,nj->ni", _rotmat(sf[L.f_quat:L.f_quat + 4].T), w)

    @property
    def rpy(self):
        """Euler angles (pb.getEulerFromQuaternion for Bullet agents, the integrated rpy for
        SimplePhysics agents)."""
        sf, L = self._fields()
        if self.physics_type == PHYS_SIMPLE:
            return sf[L.f_rpy:L.f_rpy + 3].T.clone(memory_format=torch.contiguous_format)
        return _euler_from_quat(sf[L.f_quat:L.f_quat + 4].T)

    def close(self):
        self.env.close()


def _rotmat(q):
    x, y, z, w = q.unbind(1)
    s = 2.0 / (x * x + y * y + z * z + w * w)
    return torch.stack([
        1 - s * (y * y + z * z), s * (x * y - w * z), s * (x * z + w * y),
        s * (x * y + w * z), 1 - s * (x * x + z * z), s * (y * z - w * x),
        s * (x * z - w * y), s * (y * z + w * x), 1 - s * (x * x + y * y)], 1).view(-1, 3, 3)


def _euler_from_quat(q):
    x, y, z, w = q.unbind(1)
    sarg = (-2.0 * (x * z - w * y)).clamp(-1.0, 1.0)
    roll = torch.atan2(2 * (y * z + w * x), w * w - x * x - y * y + z * z)
    pitch = torch.asin(sarg)
    yaw = torch.atan2(2 * (x * y + w * z), w * w + x * x - y * y - z * z)
    return torch.stack([roll, pitch, yaw], 1)


class BasePhysics:
    """envs/physics.py:8-76.  ``PHYSICS``: the cf2 physics type the class runs (None: the drone's)."""

    PHYSICS: int | None = None
    TAKES_DSTB = False

    def __init__(self, drone: BatchedDrone, bc=None, time_step: float | None = None, gravity: float = 9.81,
                 number_solver_iterations: int = 5, use_ground_effect: bool = False):
        if not isinstance(drone, BatchedDrone):
            raise TypeError("drone must be a cf2sim.physics.BatchedDrone (the batched agents the kernel steps)")
        if self.PHYSICS is not None and drone.physics_type != self.PHYSICS:
            raise ValueError(f"{type(self).__name__} needs a {'cf21x_bullet' if self.PHYSICS == PHYS_BULLET else 'cf21x_sys_eq'}"
                             f" drone, got {drone.drone_model} (the kernel keeps their states in different forms)")
        if use_ground_effect and drone.physics_type != PHYS_BULLET:
            raise ValueError("ground effect needs Bullet physics (SimplePhysics has none, physics.py:130-200)")
        if abs(float(gravity) - float(drone.env.cfg.gravity_world)) > 1e-12:
            raise NotImplementedError("gravity is fixed by the drone's configuration (9.81)")
        self.drone = drone
        self.bc = bc
        self.G = gravity
        self.use_ground_effect = use_ground_effect
        self.time_step = time_step
        self.number_solver_iterations = number_solver_iterations
        self._lib = _native.load()
        if drone.physics_type == PHYS_BULLET:
            # calculate_ground_effect (physics.py:27-58) in the kernel's sub-step when enabled
            _native.check(self._lib.cf2_set_ground_effect(drone.env._ctx, int(bool(use_ground_effect))),
                          "cf2_set_ground_effect")

    def set_parameters(self, time_step: float | None, number_solver_iterations: int):
        """physics.py:60-68.  ``time_step=None``: every drone integrates with its own per-episode
        dt (domain randomisation, envs/base.py:262-267); a float: all drones use it.  The solver
        iteration count has no effect: the restated multibody step has no contact constraints."""
        if time_step is not None and not 0.0 < float(time_step) < 1.0:
            raise ValueError("time_step must be in (0, 1) s")
        self.time_step = time_step
        self.number_solver_iterations = number_solver_iterations

    def _launch(self, action, dstb):
        env = self.drone.env
        a = action
        if not isinstance(a, torch.Tensor):
            a = torch.as_tensor(a, dtype=torch.float32)
        if a.dim() == 1:
            a = a.view(1, -1)
        a = a.to(device=env.device, dtype=torch.float32).contiguous()
        if a.shape != (env.num_envs, 4):
            raise ValueError(f"action must be [{env.num_envs}, 4], got {tuple(a.shape)}")
        if a.data_ptr() % 16:
            a = a.clone()
        d = None
        if dstb is not None:
            d = torch.as_tensor(dstb, dtype=torch.float32).to(env.device).contiguous()
            if d.dim() == 1:
                d = d.view(1, -1)
            if d.shape != (env.num_envs, 3):
                raise ValueError(f"dstb must be [{env.num_envs}, 3], got {tuple(d.shape)}")
        dt = 0.0 if self.time_step is None else float(self.time_step)
        _native.check(self._lib.cf2_physics_step(env._ctx, a.data_ptr(), _native.ptr(d), ctypes.c_float(dt),
                                                 env.stream), "cf2_physics_step")
        env._state_version += 1

    def step_forward(self, action, *args, **kwargs) -> None:
        raise NotImplementedError


class PyBulletPhysics(BasePhysics):
    """physics.py:79-124: motor forces, yaw torque and drag; no adversary torques."""
    PHYSICS = PHYS_BULLET

    def step_forward(self, action, *args, **kwargs) -> None:
        self._launch(action, None)


class PybulletPhysicsWithAdversary(BasePhysics):
    """physics.py:202-250: as PyBulletPhysics plus the adversary torques dstb[:, 0], dstb[:, 1]
    (dstb[:, 2] is not applied, physics.py:228-229)."""
    PHYSICS = PHYS_BULLET
    TAKES_DSTB = True

    def step_forward(self, action, dstb, *args, **kwargs) -> None:
        self._launch(action, dstb)


class SimplePhysics(BasePhysics):
    """physics.py:127-200: the system difference equations of the cf21x_sys_eq agent."""
    PHYSICS = PHYS_SIMPLE

    def step_forward(self, action, *args, **kwargs) -> None:
        self._launch(action, None)


class HipBatchedPhysics(BasePhysics):
    """The drone's own physics (Bullet restatement or SimplePhysics), adversary torques applied when
    given (Bullet drones)."""
    PHYSICS = None
    TAKES_DSTB = True

    def step_forward(self, action, dstb=None, *args, **kwargs) -> None:
        if dstb is not None and self.drone.physics_type == PHYS_SIMPLE:
            raise ValueError("SimplePhysics takes no disturbance torques (physics.py:130-200)")
        self._launch(action, dstb)
