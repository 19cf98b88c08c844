"""Env configuration: robot constants, per-env-id task flavour, and the cf2_config mirror.

This is the host-side half of the reference's agent/env constructors:

* ``RobotParams.from_urdf`` mirrors ``CrazyFlieAgent._parse_robot_parameters``
  (envs/agents.py:226-257) and the derived constants of ``CrazyFlieAgent.__init__``
  (envs/agents.py:142-206).
* ``ENV_SPECS`` mirrors the constructor defaults of every hover env class
  (envs/base.py:26-155, envs/hover.py, envs/hover_free.py) so that one C struct
  (``include/cf2sim.h: cf2_config``) describes an env id completely.

All constants are computed in float64 exactly as the reference computes them; the HIP
kernel receives them once and converts to fp32.
"""
from __future__ import annotations

import ctypes
import dataclasses
import math
import os
import xml.etree.ElementTree as etxml

import numpy as np

ASSETS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "assets")

# enums (include/cf2sim.h)
PHYS_BULLET, PHYS_SIMPLE = 0, 1
TASK_HOVER, TASK_HOVER_FREE = 0, 1
DSTB_NONE, DSTB_EXTERNAL, DSTB_UNIFORM, DSTB_CONST, DSTB_GUST, DSTB_HJ = range(6)
LEVEL_FIXED, LEVEL_BOLTZMANN = 0, 1
HJ_PTS = 15
NUM_LEVELS_MAX = 32

_d = ctypes.c_double
_i = ctypes.c_int32


class CF2Config(ctypes.Structure):
    """Field-for-field mirror of ``cf2_config`` (include/cf2sim.h)."""

    _fields_ = [
        ("num_envs", ctypes.c_uint32), ("env_id_offset", ctypes.c_uint32), ("seed", ctypes.c_uint64),
        ("physics", _i), ("task", _i), ("disturbance", _i), ("level_mode", _i),
        ("aggregate_phy_steps", _i), ("obs_rate", _i), ("buf_size", _i), ("use_latency", _i),
        ("use_motor_dynamics", _i), ("max_episode_steps", _i), ("auto_reset", _i),
        ("enable_reset_distribution", _i), ("observation_noise_on", _i), ("domain_randomization_on", _i),
        ("domain_randomization", _d), ("motor_thrust_noise", _d),
        ("sim_freq", _d), ("time_step", _d),
        ("mass", _d), ("arm", _d), ("thrust2weight", _d), ("ixx", _d), ("iyy", _d), ("izz", _d),
        ("drag_xy", _d), ("drag_z", _d), ("gravity_agent", _d), ("gravity_world", _d),
        ("motor_time_constant", _d), ("ft0", _d), ("ft1", _d), ("K", _d), ("A", _d), ("B", _d),
        ("hover_x", _d), ("hover_action", _d), ("prop_mass", _d), ("prop_inertia", _d),
        ("prop_xy", _d), ("prop_z", _d), ("prop_speed_gain", _d), ("lin_damping", _d),
        ("ang_damping", _d), ("max_coord_velocity", _d),
        ("init_xyz", _d * 3), ("reset_pos_lim", _d), ("reset_angle_lim", _d), ("reset_yaw_lim", _d),
        ("reset_vel_lim", _d), ("reset_rate_lim", _d), ("reset_yaw_rate_lim", _d),
        ("action_init_std", _d), ("motor_init_std", _d),
        ("pos_norm_std", _d), ("pos_unif_range", _d), ("vel_norm_std", _d), ("vel_unif_range", _d),
        ("rot_norm_std", _d), ("rot_unif_range", _d), ("gyro_noise_density", _d),
        ("gyro_random_walk", _d), ("gyro_bias_corr_time", _d), ("gyro_turn_on_bias_sigma", _d),
        ("lpf_gain", _d), ("lpf_ratio", _d),
        ("penalty_action", _d), ("penalty_angle", _d), ("penalty_spin", _d), ("penalty_terminal", _d),
        ("penalty_velocity", _d), ("penalty_z", _d), ("penalty_arp", _d), ("penalty_dist", _d),
        ("target_pos", _d * 3), ("target_rpy", _d * 3), ("target_rate", _d * 3),
        ("done_rp_limit", _d), ("done_rate_limit_deg", _d), ("done_z_min", _d),
        ("cost_xy_lim", _d), ("cost_z_lim", _d), ("cost_rp_lim", _d), ("cost_vel_lim", _d),
        ("cost_rate_lim", _d),
        ("dstb_level", _d), ("dstb_umax", _d * 3), ("dstb_uniform_hi", _d * 3),
        ("gust_onset_prob", _d), ("gust_max_level", _d), ("gust_duration", _i), ("num_levels", _i),
        ("level_values", _d * NUM_LEVELS_MAX), ("level_cdf", _d * NUM_LEVELS_MAX),
        ("hj_grid_min", _d * 6), ("hj_grid_dx", _d * 6), ("hj_grid_points", (_d * HJ_PTS) * 6),
        ("num_drones", _i), ("downwash_on", _i), ("dw_coeff", _d * 3), ("prop_radius", _d),
        ("formation_dx", _d), ("formation_dz", _d),
        ("use_ground_effect", _i), ("gnd_eff_coeff", _d), ("gnd_eff_h_clip", _d),
    ]

    def to_dict(self) -> dict:
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            if isinstance(v, ctypes.Array):
                v = np.ctypeslib.as_array(v).tolist()
            out[name] = v
        return out


def deg2rad(x):
    """envs/utils.py:47-49"""
    return np.pi * x / 180


@dataclasses.dataclass
class RobotParams:
    """Constants parsed from a URDF as ``CrazyFlieAgent._parse_robot_parameters`` does."""

    M: float
    L: float
    THRUST2WEIGHT_RATIO: float
    IXX: float
    IYY: float
    IZZ: float
    KF: float
    KM: float
    DRAG_COEFF_XY: float
    DRAG_COEFF_Z: float
    GND_EFF_COEFF: float
    PROP_RADIUS: float
    DW_COEFF_1: float
    DW_COEFF_2: float
    DW_COEFF_3: float
    prop_mass: float = 0.0
    prop_inertia: float = 0.0
    prop_xy: float = 0.028
    prop_z: float = 0.0

    @classmethod
    def from_urdf(cls, file_name: str) -> "RobotParams":
        path = file_name if os.path.isabs(file_name) else os.path.join(ASSETS, file_name)
        root = etxml.parse(path).getroot()
        props = root.find("properties").attrib
        base = root.find("link[@name='base_link']/inertial")
        inertia = base.find("inertia").attrib
        kw = dict(
            M=float(base.find("mass").attrib["value"]),
            L=float(props["arm"]),
            THRUST2WEIGHT_RATIO=float(props["thrust2weight"]),
            IXX=float(inertia["ixx"]), IYY=float(inertia["iyy"]), IZZ=float(inertia["izz"]),
            KF=float(props["kf"]), KM=float(props["km"]),
            DRAG_COEFF_XY=float(props["drag_coeff_xy"]), DRAG_COEFF_Z=float(props["drag_coeff_z"]),
            GND_EFF_COEFF=float(props["gnd_eff_coeff"]), PROP_RADIUS=float(props["prop_radius"]),
            DW_COEFF_1=float(props["dw_coeff_1"]), DW_COEFF_2=float(props["dw_coeff_2"]),
            DW_COEFF_3=float(props["dw_coeff_3"]),
        )
        prop = root.find("link[@name='m1_link']/inertial")
        joint = root.find("joint[@name='prop1_joint']/origin")
        if prop is not None and joint is not None:
            kw["prop_mass"] = float(prop.find("mass").attrib["value"])
            kw["prop_inertia"] = float(prop.find("inertia").attrib["izz"])
            xyz = [float(s) for s in joint.attrib["xyz"].split()]
            kw["prop_xy"] = abs(xyz[0])
            kw["prop_z"] = xyz[2]
        return cls(**kw)


@dataclasses.dataclass
class EnvSpec:
    """Constructor defaults of one reference env class."""

    cls_name: str
    module: str                 # 'hover' or 'hover_free'
    physics: int
    task: int
    disturbance: int
    urdf: str = "cf21x_bullet.urdf"
    sim_freq: int = 200
    aggregate_phy_steps: int = 2
    observation_frequency: int = 100
    use_latency: bool = True
    use_motor_dynamics: bool = True
    level_mode: int = LEVEL_FIXED
    disturbance_level: float = 0.0
    done_rp_deg: float = 60.0
    done_rate_deg: float = 300.0
    initial_angle: float = np.pi / 6
    reset_rate_deg: float = 200.0    # DroneHover*EnvWithAdversaryInitial: deg2rad(300) (rpy_dot_limit)
    registered_id: str | None = None
    num_drones: int = 1              # drones per env group (multi-drone extension, BASELINE config 5)
    downwash: bool = False


def _hover_specs():
    specs = {}

    def add(spec):
        specs[spec.cls_name] = spec

    # envs/hover.py
    add(EnvSpec("DroneHoverSimpleEnv", "hover", PHYS_SIMPLE, TASK_HOVER, DSTB_NONE, urdf="cf21x_sys_eq.urdf",
                sim_freq=100, aggregate_phy_steps=1, use_latency=False, use_motor_dynamics=False,
                registered_id="DroneHoverSimpleEnv-v0"))
    add(EnvSpec("DroneHoverBulletEnv", "hover", PHYS_BULLET, TASK_HOVER, DSTB_NONE,
                registered_id="DroneHoverBulletEnv-v0"))
    adv = dict(done_rp_deg=75.0, done_rate_deg=1000.0)
    for task, mod, prefix in ((TASK_HOVER, "hover", "DroneHoverBulletEnv"),
                              (TASK_HOVER_FREE, "hover_free", "DroneHoverBulletFreeEnv")):
        add(EnvSpec(prefix + "WithAdversary", mod, PHYS_BULLET, task, DSTB_HJ,
                    disturbance_level=0.0 if task == TASK_HOVER else 1.5, **adv))
        add(EnvSpec(prefix + "WithRandomHJAdversary", mod, PHYS_BULLET, task, DSTB_HJ,
                    level_mode=LEVEL_BOLTZMANN, **adv))
        add(EnvSpec(prefix + "WithoutAdversary", mod, PHYS_BULLET, task, DSTB_NONE, **adv))
        add(EnvSpec(prefix + "WithRandomAdversary", mod, PHYS_BULLET, task, DSTB_UNIFORM, **adv))
        add(EnvSpec(prefix + "WithAdversaryInitial", mod, PHYS_BULLET, task, DSTB_HJ, disturbance_level=1.5,
                    initial_angle=np.pi / 4, reset_rate_deg=300.0, **adv))
        add(EnvSpec(prefix + "WithCurriculumHJAdversary", mod, PHYS_BULLET, task, DSTB_HJ,
                    level_mode=LEVEL_BOLTZMANN, **adv))
        # build-defined workloads of BASELINE.json (not reference classes)
        add(EnvSpec(prefix + "WithConstWind", mod, PHYS_BULLET, task, DSTB_CONST, disturbance_level=1.0, **adv))
        add(EnvSpec(prefix + "WithGust", mod, PHYS_BULLET, task, DSTB_GUST, disturbance_level=1.5, **adv))
        if task == TASK_HOVER_FREE:   # position-free reward: formations need no per-drone target
            # BASELINE config 5: 4-drone formations with downwash + the per-step stochastic torque
            add(EnvSpec(prefix + "WithDownwash", mod, PHYS_BULLET, task, DSTB_UNIFORM, num_drones=4,
                        downwash=True, **adv))
    for name in ("WithAdversary", "WithRandomHJAdversary", "WithoutAdversary", "WithRandomAdversary",
                 "WithAdversaryInitial", "WithCurriculumHJAdversary"):
        specs["DroneHoverBulletEnv" + name].registered_id = "DroneHoverBulletEnv" + name + "-v0"
    for name in ("WithoutAdversary", "WithAdversary", "WithRandomHJAdversary"):
        specs["DroneHoverBulletFreeEnv" + name].registered_id = "DroneHoverBulletFreeEnv" + name + "-v0"
    for name in ("WithConstWind", "WithGust", "WithDownwash"):   # extensions, under their own ids
        for prefix in ("DroneHoverBulletEnv", "DroneHoverBulletFreeEnv"):
            if prefix + name in specs:
                specs[prefix + name].registered_id = prefix + name + "-v0"
    return specs


ENV_SPECS = _hover_specs()
# the 12 hover ids of the reference registry (phoenix_drone_simulation/__init__.py:8-109)
EXTENSION_KEYS = ("ConstWind", "Gust", "Downwash")
REFERENCE_IDS = [s.registered_id for s in ENV_SPECS.values()
                 if s.registered_id and not any(k in s.registered_id for k in EXTENSION_KEYS)]
# registered by the reference but outside the accelerated hover path
OUT_OF_SCOPE_IDS = ["DroneTakeOffSimpleEnv-v0", "DroneTakeOffBulletEnv-v0",
                    "DroneCircleSimpleEnv-v0", "DroneCircleBulletEnv-v0"]


def spec_for_id(env_id: str) -> EnvSpec:
    """Resolve a registered id ('DroneHoverBulletFreeEnvWithAdversary-v0'), any hover class name
    with or without '-v0' (e.g. the unregistered 'DroneHoverBulletFreeEnvWithRandomAdversary')."""
    for s in ENV_SPECS.values():
        if s.registered_id == env_id:
            return s
    name = env_id[:-3] if env_id.endswith("-v0") else env_id
    if name in ENV_SPECS:
        return ENV_SPECS[name]
    if env_id in OUT_OF_SCOPE_IDS:
        raise NotImplementedError(f"{env_id}: take-off / circle tasks are outside the accelerated hover path "
                                  "(see DESIGN.md 'Out of scope')")
    raise KeyError(f"unknown env id {env_id!r}")


def boltzmann_table(low=0.0, high=2.1, accuracy=0.1):
    """Support and normalised CDF of ``Boltzmann()`` envs/utils.py:27-39 as numpy's
    ``choice(p=...)`` uses them (cdf = cumsum(p); cdf /= cdf[-1]; searchsorted(u, 'right'))."""
    energies = np.array(np.arange(low, high, accuracy))
    weights = np.exp(-1.0 * energies)
    p = weights / np.sum(weights)
    cdf = p.cumsum()
    cdf /= cdf[-1]
    values = np.around(energies, 1)
    return values, cdf


def hj_grid():
    """Grid(...) of distur_gener.py:179 with GridProcessing.Grid.__init__ (:6-49) semantics."""
    gmin = np.array([-math.pi / 2.4, -math.pi / 2.4, -math.pi / 2.4, -math.pi, -math.pi, -math.pi])
    gmax = np.array([math.pi / 2.4, math.pi / 2.4, math.pi / 2.4, math.pi, math.pi, math.pi])
    pts = np.array([15, 15, 15, 15, 15, 15])
    for dim in (0, 1, 2):  # periodic dims exclude the upper bound
        gmax[dim] = gmin[dim] + (gmax[dim] - gmin[dim]) * (1 - 1 / pts[dim])
    dx = (gmax - gmin) / (pts - 1.0)
    points = [np.linspace(gmin[i], gmax[i], num=pts[i]) for i in range(6)]
    return gmin, dx, points


def build_config(env_id_or_spec, num_envs: int, seed: int = 0, env_id_offset: int = 0,
                 auto_reset: bool = True, **kwargs) -> CF2Config:
    """Fill a cf2_config for ``num_envs`` copies of an env id, honouring the reference's
    constructor kwargs (observation_noise, domain_randomization, motor_thrust_noise,
    latency, motor_time_constant, enable_reset_distribution, aggregate_phy_steps,
    penalty_*, disturbance_level, max_episode_steps ...)."""
    spec = env_id_or_spec if isinstance(env_id_or_spec, EnvSpec) else spec_for_id(env_id_or_spec)
    kw = dict(kwargs)
    robot = RobotParams.from_urdf(spec.urdf)
    c = CF2Config()
    c.num_envs = int(num_envs)
    c.env_id_offset = int(env_id_offset)
    c.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    c.physics = spec.physics
    c.task = spec.task
    c.disturbance = kw.pop("disturbance", spec.disturbance)
    c.level_mode = spec.level_mode

    sim_freq = kw.pop("sim_freq", spec.sim_freq)
    agg = kw.pop("aggregate_phy_steps", spec.aggregate_phy_steps)
    obs_freq = kw.pop("observation_frequency", spec.observation_frequency)
    latency = kw.pop("latency", 0.015)
    mtc = kw.pop("motor_time_constant", 0.080)
    thrust_noise = kw.pop("motor_thrust_noise", 0.05)
    obs_noise = kw.pop("observation_noise", 1)
    dr = kw.pop("domain_randomization", 0.10)
    hist = kw.pop("observation_history_size", 2)
    if hist != 2:
        raise NotImplementedError("observation_history_size != 2 is not implemented by the HIP kernel")
    time_step = 1.0 / sim_freq                                   # base.py:96
    c.sim_freq = float(sim_freq)
    c.time_step = time_step
    c.aggregate_phy_steps = int(agg)
    c.obs_rate = int(sim_freq // obs_freq)                       # base.py:106
    use_latency = spec.use_latency if latency >= time_step else False   # agents.py:165
    c.use_latency = int(use_latency)
    c.buf_size = int(max(1, int(latency // time_step)))          # agents.py:180
    if c.buf_size > 4:
        raise NotImplementedError("latency ring longer than 4 sub-steps")
    c.use_motor_dynamics = int(spec.use_motor_dynamics)
    c.max_episode_steps = int(kw.pop("max_episode_steps", 500))
    c.auto_reset = int(auto_reset)
    c.enable_reset_distribution = int(kw.pop("enable_reset_distribution", True))
    c.observation_noise_on = int(obs_noise > 0)
    c.domain_randomization_on = int(dr > 0)
    c.domain_randomization = float(dr)
    c.motor_thrust_noise = float(thrust_noise)

    # robot (agents.py:142-206)
    G = 9.81
    c.mass, c.arm, c.thrust2weight = robot.M, robot.L, robot.THRUST2WEIGHT_RATIO
    c.ixx, c.iyy, c.izz = robot.IXX, robot.IYY, robot.IZZ
    c.drag_xy, c.drag_z = robot.DRAG_COEFF_XY, robot.DRAG_COEFF_Z
    c.gravity_agent = G
    c.gravity_world = 9.81                                       # base.py:192, physics.py:16
    c.motor_time_constant = mtc
    c.ft0, c.ft1 = 1.56e-5, 5.96e-3
    gravity = G * robot.M
    max_thrust = gravity * robot.THRUST2WEIGHT_RATIO / 4
    c.K = max_thrust
    c.A = 1 - time_step / mtc
    c.B = time_step / mtc
    c.hover_x = float(np.sqrt(1 / robot.THRUST2WEIGHT_RATIO))
    c.hover_action = 2 * 1 / robot.THRUST2WEIGHT_RATIO - 1
    c.prop_mass, c.prop_inertia = robot.prop_mass, robot.prop_inertia
    c.prop_xy, c.prop_z = robot.prop_xy, robot.prop_z
    c.prop_speed_gain = 100.0
    c.lin_damping = c.ang_damping = 0.04
    c.max_coord_velocity = 100.0

    # reset distribution (hover_free.py:237-289 / hover.py:204-256 / *AdversaryInitial)
    for k, v in enumerate((0.0, 0.0, 1.0)):
        c.init_xyz[k] = v
    c.reset_pos_lim = 0.25
    c.reset_angle_lim = float(spec.initial_angle)
    c.reset_yaw_lim = 2 * np.pi
    c.reset_vel_lim = 0.1
    c.reset_rate_lim = float(deg2rad(spec.reset_rate_deg))
    c.reset_yaw_rate_lim = float(deg2rad(20))
    c.action_init_std = 0.02
    c.motor_init_std = 0.02

    # SensorNoise defaults (sensors.py:17-33) and the gyro LPF (base.py:107-108)
    c.pos_norm_std, c.pos_unif_range = 0.002, 0.001
    c.vel_norm_std, c.vel_unif_range = 0.01, 0.0
    c.rot_norm_std, c.rot_unif_range = float(deg2rad(0.1)), float(deg2rad(0.05))
    c.gyro_noise_density, c.gyro_random_walk = 0.000175, 0.0105
    c.gyro_bias_corr_time, c.gyro_turn_on_bias_sigma = 1000.0, float(deg2rad(5))
    lpf_T, lpf_Ts = 2 / sim_freq, 1 / sim_freq
    c.lpf_gain, c.lpf_ratio = 1.0, lpf_Ts / lpf_T

    # reward / done / cost
    if spec.task == TASK_HOVER:          # hover.py:16-34, 184-202
        pen = dict(penalty_action=1e-4, penalty_angle=0.0, penalty_spin=1e-4, penalty_terminal=1000.0,
                   penalty_velocity=0.0, penalty_z=0.0)
        c.penalty_dist = 1.0
    else:                                # hover_free.py:17-38, 206-235
        pen = dict(penalty_action=0.0, penalty_angle=1.0, penalty_spin=1.0, penalty_terminal=1000.0,
                   penalty_velocity=1.0, penalty_z=0.0)
        c.penalty_dist = 0.0
    for k in list(pen):
        pen[k] = float(kw.pop(k, pen[k]))
        setattr(c, k, pen[k])
    c.penalty_arp = 0.0
    tp = kw.pop("target_pos", (0.0, 0.0, 1.0))
    for k in range(3):
        c.target_pos[k] = float(tp[k])
        c.target_rpy[k] = 0.0
        c.target_rate[k] = 0.0
    c.done_rp_limit = float(deg2rad(spec.done_rp_deg))
    c.done_rate_limit_deg = float(spec.done_rate_deg)
    c.done_z_min = 0.2
    c.cost_xy_lim, c.cost_z_lim = 0.10, 1.20
    c.cost_rp_lim = float(deg2rad(10))
    c.cost_vel_lim = 0.25
    c.cost_rate_lim = float(deg2rad(spec.reset_rate_deg))   # self.rpy_dot_limit

    # disturbance
    c.dstb_level = float(kw.pop("disturbance_level", spec.disturbance_level))
    for k, v in enumerate((5.3 * 10 ** -3, 5.3 * 10 ** -3, 1.43 * 10 ** -4)):   # distur_gener.py:152
        c.dstb_umax[k] = v
    for k, v in enumerate((1 * 10 ** -3, 1 * 10 ** -3, 1 * 10 ** -4)):         # hover_free.py:315
        c.dstb_uniform_hi[k] = v
    c.gust_onset_prob = float(kw.pop("gust_onset_prob", 0.01))
    c.gust_max_level = float(kw.pop("gust_max_level", 1.5))
    c.gust_duration = int(kw.pop("gust_duration", 20))
    values, cdf = boltzmann_table()
    c.num_levels = len(values)
    for k in range(len(values)):
        c.level_values[k] = float(values[k])
        c.level_cdf[k] = float(cdf[k])
    gmin, dx, points = hj_grid()
    for d in range(6):
        c.hj_grid_min[d] = float(gmin[d])
        c.hj_grid_dx[d] = float(dx[d])
        for k in range(HJ_PTS):
            c.hj_grid_points[d][k] = float(points[d][k])
    # multi-drone formation + downwash (extension; gym-pybullet-drones' _downwash formula with the
    # URDF coefficients the reference parses but never uses, agents.py:251-257)
    c.num_drones = int(kw.pop("num_drones", spec.num_drones))
    c.downwash_on = int(bool(kw.pop("downwash", spec.downwash)))
    c.dw_coeff[0], c.dw_coeff[1], c.dw_coeff[2] = robot.DW_COEFF_1, robot.DW_COEFF_2, robot.DW_COEFF_3
    c.prop_radius = robot.PROP_RADIUS
    c.formation_dx = float(kw.pop("formation_dx", 0.5))
    c.formation_dz = float(kw.pop("formation_dz", 1.0))
    # ground effect (BasePhysics.calculate_ground_effect physics.py:27-58; off in every reference env)
    c.use_ground_effect = int(bool(kw.pop("use_ground_effect", False)))
    c.gnd_eff_coeff = robot.GND_EFF_COEFF
    max_thrust = robot.M * 9.81 * robot.THRUST2WEIGHT_RATIO / 4.0                 # agents.py:151
    max_rpm = math.sqrt((robot.THRUST2WEIGHT_RATIO * robot.M * 9.81) / (4.0 * max_thrust))   # agents.py:155
    c.gnd_eff_h_clip = 0.25 * robot.PROP_RADIUS * math.sqrt(
        (15.0 * max_rpm ** 2 * robot.KF * robot.GND_EFF_COEFF) / max_thrust)     # agents.py:156
    if c.num_drones not in (1, 2, 4, 8):
        raise ValueError("num_drones must be 1, 2, 4 or 8")
    if c.num_envs % c.num_drones or c.env_id_offset % c.num_drones:
        raise ValueError("num_envs and env_id_offset must be multiples of num_drones (whole formations)")
    if kw:
        raise TypeError(f"unsupported env kwargs: {sorted(kw)}")
    return c


def obs_dim(cfg: CF2Config) -> int:
    """observation_space size: H * (obs + act_dim) (base.py:141)."""
    return 2 * ((13 if cfg.observation_noise_on else 17) + 4)
