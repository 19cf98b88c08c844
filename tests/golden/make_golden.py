"""Generate golden vectors by running the REFERENCE's own Python (read from /root/reference) in
this container.  Run once where /root/reference exists; the outputs (tests/golden/*.npz, data
only) are committed and the tests never read the reference at run time.

The reference imports pybullet / gym / heterocl, none of which exist here.  They are replaced by
small stand-ins defined below:
  * gym: Env base class, spaces.Box, envs.registration.register (no behaviour).
  * pybullet: the constants the env modules use and restated PyBullet C-API formulas
    (getQuaternionFromEuler, getEulerFromQuaternion, getMatrixFromQuaternion).
  * pybullet_utils.bullet_client.BulletClient: a fake physics server.  It records the forces and
    torques the reference applies, holds the base state, and advances it in stepSimulation()
    with a numpy restatement of the btMultiBody step (the same algorithm oracle/cf2_oracle.c
    restates; bullet3 itself is not available).  Everything else the env does (apply_action,
    PWM, latency, drag, force/torque assembly, update_information, sensor noise, history,
    reward/done/info, reset distribution) is the reference's own code.
  * heterocl / plotly / odp: import-only stand-ins for distur_gener.py; odp.Grid is the
    reference's GridProcessing.py loaded from its file.

Fixtures written:
  golden_env_trajectories.npz  noise-free env rollouts (Bullet free/hover, Simple) driven by
                               real-flight PWM logs, with the initial state captured after reset
  golden_components.npz        apply_action (OU draws recorded), SensorNoise.add_noise (draws
                               recorded), quaternion conversions, Boltzmann probabilities
  golden_hj.npz                distur_gener() on a synthetic (exactly reproducible) value table
  golden_env_hj_trajectories.npz  noise-free rollouts of the HJ-adversary envs (fixed level, hover
                               and hover_free, and the Boltzmann-level env) on the synthetic table
  golden_env_uniform_trajectories.npz  noise-free rollouts of the uniform-random-adversary envs
                               with every sampled dstb recorded
  golden_reset_samples.npz     3000 draws of the reference's reset distribution (pose, velocities,
                               motor state, action ring, domain-randomised parameters) for four
                               env classes, and the Boltzmann env's redrawn levels
  golden_ground_effect.npz     PyBulletPhysics(use_ground_effect=True).step_forward sub-steps of the
                               reference's drone placed near the ground (one case tilted past pi/2)
"""
from __future__ import annotations

import contextlib
import glob
import importlib.util
import math
import os
import sys
import tempfile
import types

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------------------
# stand-ins
# ----------------------------------------------------------------------------------------
def quat_from_euler(rpy):
    phi, the, psi = rpy[0] / 2.0, rpy[1] / 2.0, rpy[2] / 2.0
    q = [math.sin(phi) * math.cos(the) * math.cos(psi) - math.cos(phi) * math.sin(the) * math.sin(psi),
         math.cos(phi) * math.sin(the) * math.cos(psi) + math.sin(phi) * math.cos(the) * math.sin(psi),
         math.cos(phi) * math.cos(the) * math.sin(psi) - math.sin(phi) * math.sin(the) * math.cos(psi),
         math.cos(phi) * math.cos(the) * math.cos(psi) + math.sin(phi) * math.sin(the) * math.sin(psi)]
    n = math.sqrt(sum(x * x for x in q))
    return tuple(x / n for x in q)


def euler_from_quat(q):
    sqx, sqy, sqz, squ = q[0] * q[0], q[1] * q[1], q[2] * q[2], q[3] * q[3]
    sarg = -2 * (q[0] * q[2] - q[3] * q[1])
    if sarg <= -0.99999:
        return (0.0, -0.5 * math.pi, 2 * math.atan2(q[0], -q[1]))
    if sarg >= 0.99999:
        return (0.0, 0.5 * math.pi, 2 * math.atan2(-q[0], q[1]))
    return (math.atan2(2 * (q[1] * q[2] + q[3] * q[0]), squ - sqx - sqy + sqz), math.asin(sarg),
            math.atan2(2 * (q[0] * q[1] + q[3] * q[2]), squ + sqx - sqy - sqz))


def matrix_from_quat(q):
    x, y, z, w = q
    d = x * x + y * y + z * z + w * w
    s = 2.0 / d
    xs, ys, zs = x * s, y * s, z * s
    wx, wy, wz = w * xs, w * ys, w * zs
    xx, xy, xz = x * xs, x * ys, x * zs
    yy, yz, zz = y * ys, y * zs, z * zs
    return (1.0 - (yy + zz), xy - wz, xz + wy, xy + wz, 1.0 - (xx + zz), yz - wx, xz - wy, yz + wx, 1.0 - (xx + yy))


class FakeBullet:
    """Physics-server stand-in: base rigid body of the cf21x multibody (see module doc)."""

    GEOM_SPHERE = 2
    COV_ENABLE_RENDERING = 0

    def __init__(self, connection_mode=None):
        self.n_bodies = 0
        self.drone = None
        self.dt = 1 / 240.0
        self.g = -9.81
        self.saved = {}

    # --- world ---
    def loadURDF(self, file, *a, **kw):
        bid = self.n_bodies
        self.n_bodies += 1
        if "cf21x" in str(file):
            self.drone = bid
            self.p = np.zeros(3); self.q = np.array([0, 0, 0, 1.0]); self.v = np.zeros(3); self.w = np.zeros(3)
            self.qd = np.zeros(4)                      # prop joint rates
            self.m, self.I = 0.030, np.array([1.33e-5, 1.33e-5, 2.64e-5])
            if "sys_eq" in str(file):
                self.m, self.I = 0.027, np.array([1.7e-5, 1.7e-5, 2.9e-5])
            self.F = []; self.T = []; self.targets = np.zeros(4)
        return bid

    def setPhysicsEngineParameter(self, fixedTimeStep=None, **kw):
        if fixedTimeStep is not None:
            self.dt = float(fixedTimeStep)

    def setGravity(self, x, y, z):
        self.g = z

    def saveState(self):
        k = len(self.saved) + 1
        self.saved[k] = (self.p.copy(), self.q.copy(), self.v.copy(), self.w.copy(), self.qd.copy())
        return k

    def restoreState(self, k):
        p, q, v, w, qd = self.saved[k]
        self.p, self.q, self.v, self.w, self.qd = p.copy(), q.copy(), v.copy(), w.copy(), qd.copy()

    def resetBasePositionAndOrientation(self, bid, posObj, ornObj):
        self.p = np.array(posObj, float); self.q = np.array(ornObj, float)

    def resetBaseVelocity(self, bid, linearVelocity=None, angularVelocity=None):
        if linearVelocity is not None:
            self.v = np.array(linearVelocity, float)
        if angularVelocity is not None:
            self.w = np.array(angularVelocity, float)

    def getBasePositionAndOrientation(self, bid):
        return tuple(self.p), tuple(self.q)

    def getBaseVelocity(self, bid):
        return tuple(self.v), tuple(self.w)

    def changeDynamics(self, bodyUniqueId, linkIndex, mass=None, localInertiaDiagonal=None, **kw):
        if mass is not None:
            self.m = float(mass)
        if localInertiaDiagonal is not None:
            self.I = np.array(localInertiaDiagonal, float)

    def getQuaternionFromEuler(self, rpy):
        return quat_from_euler(rpy)

    def getEulerFromQuaternion(self, q):
        return euler_from_quat(q)

    def getMatrixFromQuaternion(self, q):
        return matrix_from_quat(q)

    def getLinkStates(self, bid, linkIndices, **kw):
        R = np.array(matrix_from_quat(self.q)).reshape(3, 3)
        offs = [(0.028, -0.028, 0.0108), (-0.028, -0.028, 0.0108), (-0.028, 0.028, 0.0108), (0.028, 0.028, 0.0108),
                (0, 0, 0)]
        return [(tuple(self.p + R @ np.array(offs[i])),) for i in linkIndices]

    # --- forces ---
    def applyExternalForce(self, bid, link, forceObj, posObj, flags):
        assert flags == 1 and list(posObj) == [0, 0, 0]          # LINK_FRAME at the link origin
        self.F.append((link, np.array(forceObj, float)))

    def applyExternalTorque(self, bid, link, torqueObj, flags):
        assert flags == 1 and link == 4
        self.T.append(np.array(torqueObj, float))

    def setJointMotorControl2(self, bodyUniqueId, jointIndex, controlMode, targetVelocity, force):
        self.targets[jointIndex] = targetVelocity

    def stepSimulation(self):
        """btMultiBody step restated (same algorithm as oracle/cf2_oracle.c bullet_substep)."""
        R = np.array(matrix_from_quat(self.q)).reshape(3, 3)
        L, Lz, mp, Ip = 0.028, 0.0108, 1e-9, 1e-9
        offs = np.array([[L, -L, Lz], [-L, -L, Lz], [-L, L, Lz], [L, L, Lz], [0, 0, 0]])
        Fb = np.zeros(3); Tb = np.zeros(3)
        for link, f in self.F:                                       # link frames == base frame
            Fb += f
            Tb += np.cross(offs[link], f)
        for t in self.T:
            Tb += t
        mtot = self.m + 4 * mp
        Fw = R @ Fb + np.array([0, 0, self.g * mtot])
        wb, vb = R.T @ self.w, R.T @ self.v
        Ic = self.I + 4 * Ip + 4 * mp * np.array([L * L + Lz * Lz, L * L + Lz * Lz, 2 * L * L])
        ax = np.array([-1.0, 1.0, -1.0, 1.0])
        sp_old, sp_new = float(ax @ self.qd), float(ax @ self.targets)
        Iw = Ic * wb + np.array([0, 0, Ip * sp_old])
        tau = Tb - np.cross(wb, Iw) - self.I * wb * 0.04 * (1 + np.linalg.norm(wb))
        for j in range(4):
            wp = wb + np.array([0, 0, ax[j] * self.qd[j]])
            tau = tau - Ip * 0.04 * (1 + np.linalg.norm(wp)) * wp
        tau[2] -= Ip * (sp_new - sp_old) / self.dt
        wdot_b = tau / Ic
        vdot = Fw / mtot - 0.04 * (1 + np.linalg.norm(vb)) * self.m / mtot * self.v
        self.w = np.clip(self.w + (R @ wdot_b) * self.dt, -100, 100)
        self.v = np.clip(self.v + vdot * self.dt, -100, 100)
        self.p = self.p + self.dt * self.v
        ang = np.linalg.norm(self.w)
        if ang * self.dt > math.pi / 4:
            ang = (math.pi / 4) / self.dt
        if ang < 0.001:
            axs = self.w * (0.5 * self.dt - self.dt ** 3 * 0.020833333333 * ang * ang)
        else:
            axs = self.w * (math.sin(0.5 * ang * self.dt) / ang)
        cw = math.cos(0.5 * ang * self.dt)
        qx, qy, qz, qw = self.q
        n = np.array([cw * qx + axs[0] * qw + axs[1] * qz - axs[2] * qy,
                      cw * qy + axs[1] * qw + axs[2] * qx - axs[0] * qz,
                      cw * qz + axs[2] * qw + axs[0] * qy - axs[1] * qx,
                      cw * qw - axs[0] * qx - axs[1] * qy - axs[2] * qz])
        self.q = n / np.linalg.norm(n)
        self.qd = self.targets.copy()
        self.F, self.T = [], []

    def __getattr__(self, name):            # rendering / debug calls: no-ops
        return lambda *a, **k: 0


def install_stubs():
    gym = types.ModuleType("gym")
    class Env:  # noqa: E306
        pass
    class Box:  # noqa: E306
        def __init__(self, low, high, shape=None, dtype=np.float32):
            self.low = np.asarray(low, dtype); self.high = np.asarray(high, dtype)
            if shape is not None:
                self.low = np.broadcast_to(self.low, shape); self.high = np.broadcast_to(self.high, shape)
            self.shape = self.low.shape; self.dtype = dtype
        def sample(self):
            return np.random.uniform(self.low, self.high).astype(self.dtype)
    gym.Env = Env
    gym.spaces = types.SimpleNamespace(Box=Box)
    reg = types.ModuleType("gym.envs.registration"); reg.register = lambda **kw: None
    envs = types.ModuleType("gym.envs"); envs.registration = reg
    sys.modules.update({"gym": gym, "gym.spaces": gym.spaces, "gym.envs": envs, "gym.envs.registration": reg})

    pb = types.ModuleType("pybullet")
    pb.LINK_FRAME, pb.WORLD_FRAME, pb.VELOCITY_CONTROL = 1, 2, 0
    pb.URDF_USE_INERTIA_FROM_FILE, pb.COV_ENABLE_GUI, pb.COV_ENABLE_RENDERING = 2, 1, 0
    pb.GUI, pb.DIRECT, pb.ER_BULLET_HARDWARE_OPENGL, pb.MAX_RAY_INTERSECTION_BATCH_SIZE = 1, 2, 131072, 16384
    pb.getQuaternionFromEuler = quat_from_euler
    pb.getEulerFromQuaternion = euler_from_quat
    pb.getMatrixFromQuaternion = matrix_from_quat
    pb.loadURDF = lambda *a, **k: -1
    sys.modules["pybullet"] = pb
    pbd = types.ModuleType("pybullet_data"); pbd.getDataPath = lambda: "/nonexistent"
    sys.modules["pybullet_data"] = pbd
    pu = types.ModuleType("pybullet_utils"); bcm = types.ModuleType("pybullet_utils.bullet_client")
    bcm.BulletClient = FakeBullet; pu.bullet_client = bcm
    sys.modules.update({"pybullet_utils": pu, "pybullet_utils.bullet_client": bcm})

    for name in ("heterocl", "plotly", "plotly.graph_objects", "odp", "odp.computeGraphs",
                 "odp.computeGraphs.CustomGraphFunctions", "odp.Shapes", "odp.Plots", "odp.solver"):
        sys.modules[name] = types.ModuleType(name)
    sys.modules["odp.computeGraphs.CustomGraphFunctions"].my_abs = abs
    sys.modules["odp.Plots"].PlotOptions = object
    sys.modules["odp.solver"].HJSolver = sys.modules["odp.solver"].TTRSolver = object
    spec = importlib.util.spec_from_file_location(
        "odp.Grid", os.path.join(REF, "phoenix_drone_simulation/adversarial_generation/odp/Grid/GridProcessing.py"))
    gridmod = importlib.util.module_from_spec(spec); spec.loader.exec_module(gridmod)
    sys.modules["odp.Grid"] = gridmod
    if REF not in sys.path:
        sys.path.insert(0, REF)


# ----------------------------------------------------------------------------------------
# fixtures
# ----------------------------------------------------------------------------------------
def flight_actions():
    """Real-flight PWM logs of the reference (experiments/07_.../logs/PWM), a = PWM/30000 - 1."""
    files = sorted(glob.glob(os.path.join(REF, "experiments/07_control_structure_hypothesis/logs/PWM/*/*/log*.csv")))
    out = []
    for f in files[:12]:
        d = np.genfromtxt(f, delimiter=",", names=True)
        a = np.stack([d["mot0"], d["mot1"], d["mot2"], d["mot3"]], 1) / 30000.0 - 1.0
        out.append(a.astype(np.float32))
    return out


def env_trajectories():
    from phoenix_drone_simulation.envs import hover, hover_free
    acts = flight_actions()
    cases = [("DroneHoverBulletFreeEnvWithoutAdversary", hover_free, {}),
             ("DroneHoverBulletEnv", hover, {}),
             ("DroneHoverBulletEnvWithoutAdversary", hover, {}),
             ("DroneHoverSimpleEnv", hover, {})]
    rec = {}
    k = 0
    for name, mod, extra in cases:
        for rep in range(3):
            np.random.seed(1000 + k)
            kw = dict(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0)
            kw.update(extra)
            env = getattr(mod, name)(**kw)
            obs0 = env.reset()
            bc, dr = env.bc, env.drone
            init = dict(p=bc.p.copy(), q=bc.q.copy(), v=bc.v.copy(), w=bc.w.copy(), x=np.array(dr.x, float),
                        abuf=np.array(dr.action_buffer, float), rpy=np.array(dr.rpy, float),
                        rpy_dot=np.array(dr.rpy_dot, float), quat=np.array(dr.quaternion, float),
                        xyz=np.array(dr.xyz, float), xyz_dot=np.array(dr.xyz_dot, float))
            a_seq = acts[k % len(acts)]
            if rep == 2 or "Simple" in name:   # near-hover random actions (SimpleEnv: no motor lag)
                a_seq = (np.random.default_rng(k).uniform(-1, 1, (50, 4)) * 0.1 + dr.HOVER_ACTION).astype(np.float32)
            O, Rw, D, C = [], [], [], []
            for a in a_seq:
                o, r, d, info = env.step(np.array(a, np.float64))
                O.append(np.array(o, float)); Rw.append(float(r)); D.append(bool(d)); C.append(float(info["cost"]))
                if d:
                    break
            key = f"{name}__{rep}"
            rec[key + "__obs0"] = np.array(obs0, float)
            for kk, vv in init.items():
                rec[key + "__init_" + kk] = vv
            rec[key + "__actions"] = np.array(a_seq[:len(O)], np.float32)
            rec[key + "__obs"] = np.array(O); rec[key + "__rew"] = np.array(Rw)
            rec[key + "__done"] = np.array(D); rec[key + "__cost"] = np.array(C)
            k += 1
    return rec


def env_hj_trajectories():
    """Noise-free rollouts of the reference's HJ-adversary envs (hover_free.py:391-444, the
    hover.py twin, and the Boltzmann-level env hover_free.py:608-683): their step() reads the
    disturbance from distur_gener (distur_gener.py:19-183), here on the synthetic value table of
    hj_vectors() saved under every level's file name.  The fixed-level envs run at level 0.5 (the
    default 1.5 flips the drone within a few env-steps); the Boltzmann env keeps its drawn level,
    which is recorded."""
    from phoenix_drone_simulation.envs import hover, hover_free
    V = synthetic_value_table()
    acts = flight_actions()
    rec = {}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        d = os.path.join(td, "phoenix_drone_simulation/adversarial_generation/FasTrack_data")
        os.makedirs(d)
        for k in range(31):
            np.save(os.path.join(d, f"fastrack_{round(0.1 * k, 1)}_15x15.npy"), V)
        os.chdir(td)
        try:
            cases = [("DroneHoverBulletFreeEnvWithAdversary", hover_free, 0.5),
                     ("DroneHoverBulletEnvWithAdversary", hover, 0.5),
                     ("DroneHoverBulletFreeEnvWithRandomHJAdversary", hover_free, None)]
            k = 0
            for name, mod, level in cases:
                for rep in range(3):
                    np.random.seed(3000 + k)
                    env = getattr(mod, name)(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0)
                    obs0 = env.reset()
                    if level is not None:
                        env.disturbance_level = level
                    bc, dr = env.bc, env.drone
                    init = dict(p=bc.p.copy(), q=bc.q.copy(), v=bc.v.copy(), w=bc.w.copy(), x=np.array(dr.x, float),
                                abuf=np.array(dr.action_buffer, float))
                    a_seq = acts[(k + 5) % len(acts)]
                    if rep == 2:
                        a_seq = (np.random.default_rng(k).uniform(-1, 1, (60, 4)) * 0.1 + dr.HOVER_ACTION).astype(np.float32)
                    O, Rw, D, C = [], [], [], []
                    for a in a_seq[:120]:
                        o, r, dn, info = env.step(np.array(a, np.float64))
                        O.append(np.array(o, float)); Rw.append(float(r)); D.append(bool(dn)); C.append(float(info["cost"]))
                        if dn:
                            break
                    key = f"{name}__{rep}"
                    rec[key + "__obs0"] = np.array(obs0, float)
                    for kk, vv in init.items():
                        rec[key + "__init_" + kk] = vv
                    rec[key + "__level"] = np.array(float(env.disturbance_level))
                    rec[key + "__actions"] = np.array(a_seq[:len(O)], np.float32)
                    rec[key + "__obs"] = np.array(O); rec[key + "__rew"] = np.array(Rw)
                    rec[key + "__done"] = np.array(D); rec[key + "__cost"] = np.array(C)
                    k += 1
        finally:
            os.chdir(cwd)
    return rec


def env_uniform_trajectories():
    """Noise-free rollouts of the reference's uniform-random-adversary envs (hover_free.py:858-1000
    and the hover.py twin :1116-1260): every env-step's dstb_space.sample() is recorded, so the
    same torques can be fed to the restatement and the kernel as external disturbances."""
    from phoenix_drone_simulation.envs import hover, hover_free
    acts = flight_actions()
    rec = {}
    k = 0
    for name, mod in (("DroneHoverBulletFreeEnvWithRandomAdversary", hover_free),
                      ("DroneHoverBulletEnvWithRandomAdversary", hover)):
        for rep in range(2):
            np.random.seed(4000 + k)
            env = getattr(mod, name)(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0)
            obs0 = env.reset()
            drawn = []
            gen = env.dstb_gen
            env.dstb_gen = lambda x, gen=gen, drawn=drawn: drawn.append(np.array(gen(x), float)) or drawn[-1]
            bc, dr = env.bc, env.drone
            init = dict(p=bc.p.copy(), q=bc.q.copy(), v=bc.v.copy(), w=bc.w.copy(), x=np.array(dr.x, float),
                        abuf=np.array(dr.action_buffer, float))
            a_seq = acts[(k + 9) % len(acts)] if rep == 0 else \
                (np.random.default_rng(k).uniform(-1, 1, (80, 4)) * 0.1 + dr.HOVER_ACTION).astype(np.float32)
            O, Rw, D, C = [], [], [], []
            for a in a_seq[:120]:
                o, r, dn, info = env.step(np.array(a, np.float64))
                O.append(np.array(o, float)); Rw.append(float(r)); D.append(bool(dn)); C.append(float(info["cost"]))
                if dn:
                    break
            key = f"{name}__{rep}"
            rec[key + "__obs0"] = np.array(obs0, float)
            for kk, vv in init.items():
                rec[key + "__init_" + kk] = vv
            rec[key + "__dstb"] = np.array(drawn)
            rec[key + "__actions"] = np.array(a_seq[:len(O)], np.float32)
            rec[key + "__obs"] = np.array(O); rec[key + "__rew"] = np.array(Rw)
            rec[key + "__done"] = np.array(D); rec[key + "__cost"] = np.array(C)
            k += 1
    return rec


def reset_samples():
    """Samples of the reference's reset distribution: DroneBaseEnv.reset (base.py:420-464) with
    task_specific_reset (hover_free.py:237-289) and apply_domain_randomization (base.py:241-298) at
    the default 10 %, repeated 3000 times; the state and per-episode parameters are recorded after
    each reset (the same public-snapshot fields the kernel's reset writes)."""
    from phoenix_drone_simulation.envs import hover, hover_free
    names = (["p0", "p1", "p2", "q0", "q1", "q2", "q3", "v0", "v1", "v2", "w0", "w1", "w2"]
             + [f"x{j}" for j in range(4)] + [f"abuf{r}{j}" for r in range(2) for j in range(4)]
             + ["dt", "m", "Jx", "Jy", "Jz", "k0", "k1"] + [f"B{j}" for j in range(4)] + [f"K{j}" for j in range(4)])
    rec = {"names": np.array(names)}
    # the default free-hover env; the hover (position-reward) twin (hover.py:204-256); the
    # AdversaryInitial variant (hover_free.py:1205-1257: pi/4 angles, 300 deg/s rates); the
    # Boltzmann-level env, whose level is redrawn at every reset (recorded as "level")
    cases = [("samples", hover_free.DroneHoverBulletFreeEnvWithoutAdversary),
             ("samples_hover", hover.DroneHoverBulletEnvWithoutAdversary),
             ("samples_initial", hover_free.DroneHoverBulletFreeEnvWithAdversaryInitial),
             ("samples_randomhj", hover_free.DroneHoverBulletFreeEnvWithRandomHJAdversary)]
    for c, (key, cls) in enumerate(cases):
        np.random.seed(5000 + c)
        env = cls()
        bc, dr = env.bc, env.drone
        rows, levels = [], []
        for _ in range(3000):
            env.reset()
            rows.append(np.concatenate([bc.p, bc.q, bc.v, bc.w, np.array(dr.x, float),
                                        np.array(dr.action_buffer, float).ravel(),
                                        [env.time_step, bc.m], bc.I,
                                        [dr.force_torque_factor_0, dr.force_torque_factor_1],
                                        np.array(dr.B, float), np.array(dr.K, float)]))
            levels.append(float(getattr(env, "disturbance_level", 0.0)))
        rec[key] = np.array(rows, np.float32)
        if key == "samples_randomhj":
            rec["levels_randomhj"] = np.array(levels)
    return rec


@contextlib.contextmanager
def recording_numpy_random(module, log):
    """Replace module.np.random.{normal,uniform,randn} by recorders that draw standard values
    and return exactly what numpy's formulas give (loc + scale*z, low + (high-low)*u)."""
    real = module.np.random
    rng = np.random.default_rng(77)

    class R:
        def normal(self, loc=0.0, scale=1.0, size=None):
            z = rng.standard_normal(size); log.append(("n", np.atleast_1d(z).copy())); return loc + scale * z
        def uniform(self, low=0.0, high=1.0, size=None):
            u = rng.random(size); log.append(("u", np.atleast_1d(u).copy())); return low + (np.asarray(high) - np.asarray(low)) * u
        def randn(self, *shape):
            z = rng.standard_normal(shape); log.append(("n", np.atleast_1d(z).copy())); return z
        def __getattr__(self, n):
            return getattr(real, n)
    saved = module.np
    module.np = types.SimpleNamespace(**{k: getattr(np, k) for k in dir(np) if not k.startswith("__")})
    module.np.random = R()
    try:
        yield
    finally:
        module.np = saved


def components():
    from phoenix_drone_simulation.envs import agents, sensors, utils
    from phoenix_drone_simulation.envs.base import DroneBaseEnv  # noqa: F401  (import check)
    from phoenix_drone_simulation.adversarial_generation.FasTrack_data.distur_gener import quat2euler
    rec = {}
    # --- apply_action with OU thrust noise, draws recorded (agents.py:259-298, utils.py:111-134) ---
    bc = FakeBullet()
    drone = agents.CrazyFlieBulletAgent(bc=bc, control_mode="PWM", time_step=0.005, aggregate_phy_steps=2,
                                        latency=0.015, motor_time_constant=0.080, motor_thrust_noise=0.05)
    drone.x = np.random.default_rng(1).normal(drone.HOVER_X, 0.02, 4)
    drone.action_buffer = np.clip(np.random.default_rng(2).normal(drone.HOVER_ACTION, 0.02, (2, 4)), -1, 1)
    rec["aa_init_x"] = drone.x.copy(); rec["aa_init_buf"] = drone.action_buffer.copy()
    acts = np.concatenate(flight_actions()[:2])[:80].astype(np.float64)
    log = []
    F, TZ, X = [], [], []
    with recording_numpy_random(utils, log):
        for a in acts:
            f, tz = drone.apply_action(a)
            F.append(np.array(f)); TZ.append(tz); X.append(drone.x.copy())
    rec["aa_actions"] = acts; rec["aa_ou_normals"] = np.array([z for _, z in log])
    rec["aa_forces"] = np.array(F); rec["aa_tz"] = np.array(TZ); rec["aa_x"] = np.array(X)
    # --- SensorNoise.add_noise with recorded draws (sensors.py:75-134) ---
    sn = sensors.SensorNoise()
    rng = np.random.default_rng(3)
    ins, outs, draws = [], [], []
    for t in range(64):
        pos, vel = rng.normal(0, 1, 3), rng.normal(0, 1, 3)
        rot = np.array([rng.uniform(-3.2, 3.2), rng.uniform(-1.6, 1.6), rng.uniform(-3.2, 3.2)])
        om = rng.normal(0, 3, 3)
        bias0 = sn.gyro_bias.copy()
        log = []
        with recording_numpy_random(sensors, log):
            p2, v2, r2, o2, _ = sn.add_noise(pos=pos, vel=vel, rot=rot, omega=om, acc=np.zeros(3), dt=1 / 200)
        z = [v for k, v in log if k == "n"]; u = [v for k, v in log if k == "u"]
        # order: pos n, vel n, bias n, rw n, turn-on n, rot n, acc n, acc n ; pos u, vel u, rot u
        normals = np.concatenate([z[0], z[1], z[2], z[3], z[4], z[5]])
        unif = np.concatenate([u[0], u[2]])
        ins.append(np.concatenate([pos, vel, rot, om, bias0])); draws.append(np.concatenate([normals, unif]))
        outs.append(np.concatenate([p2, v2, r2, o2, sn.gyro_bias]))
    rec["sn_in"] = np.array(ins); rec["sn_draws"] = np.array(draws); rec["sn_out"] = np.array(outs)
    # --- quaternion conversions (utils.py:58-82, distur_gener.py:186-207) ---
    rpy = np.random.default_rng(4).uniform(-2, 2, (256, 3))
    rec["q_rpy"] = rpy
    rec["q_utils"] = np.array([utils.get_quaternion_from_euler(r) for r in rpy])
    qs = np.random.default_rng(5).normal(size=(256, 4)); qs /= np.linalg.norm(qs, axis=1, keepdims=True)
    rec["q_quats"] = qs
    rec["q_quat2euler"] = np.array([quat2euler(q) for q in qs])
    # --- Boltzmann level distribution (utils.py:27-39): capture the p handed to np.random.choice ---
    captured = {}
    real_choice = np.random.choice
    def choice(a, p=None):
        captured["a"], captured["p"] = np.array(a), np.array(p)
        return real_choice(a, p=p)
    utils.np.random.choice = choice
    try:
        utils.Boltzmann()
    finally:
        utils.np.random.choice = real_choice
    rec["boltz_energies"] = captured["a"]; rec["boltz_p"] = captured["p"]
    return rec


def ground_effect_trajectories():
    """PyBulletPhysics(use_ground_effect=True).step_forward (physics.py:27-58, 91-124) driven on the
    reference's own drone near the ground: the env is built and reset as usual, then the base is
    placed low (tilted, moving) and the reference's physics object, constructed with ground
    effect on, is stepped directly; the state is recorded after every sub-step."""
    from phoenix_drone_simulation.envs import hover_free, physics
    rec = {}
    for k in range(4):
        np.random.seed(2000 + k)
        env = hover_free.DroneHoverBulletFreeEnvWithoutAdversary(observation_noise=0, domain_randomization=-1,
                                                                motor_thrust_noise=0)
        env.reset()
        bc, dr = env.bc, env.drone
        rng = np.random.default_rng(50 + k)
        p = np.array([rng.uniform(-0.5, 0.5), rng.uniform(-0.5, 0.5), [0.005, 0.03, 0.08, 0.2][k]])
        rpy = rng.uniform(-0.3, 0.3, 3) if k < 3 else np.array([0.2, 2.0, 0.1])   # k=3: |pitch| > pi/2
        bc.resetBasePositionAndOrientation(dr.body_unique_id, p, quat_from_euler(rpy))
        bc.resetBaseVelocity(dr.body_unique_id, rng.normal(0, 0.2, 3), rng.normal(0, 1.0, 3))
        dr.update_information()
        phys = physics.PyBulletPhysics(dr, bc, time_step=env.time_step, use_ground_effect=True)
        key = f"ge__{k}"
        rec[key + "__init_p"] = bc.p.copy(); rec[key + "__init_q"] = bc.q.copy()
        rec[key + "__init_v"] = bc.v.copy(); rec[key + "__init_w"] = bc.w.copy()
        rec[key + "__init_x"] = np.array(dr.x, float); rec[key + "__init_abuf"] = np.array(dr.action_buffer, float)
        acts = (rng.uniform(-1, 1, (120, 4)) * 0.15 + dr.HOVER_ACTION).astype(np.float32)
        S = []
        for a in acts:
            phys.step_forward(np.array(a, np.float64))
            S.append(np.concatenate([bc.p, bc.q, bc.v, bc.w, np.array(dr.x, float)]))
        rec[key + "__actions"] = acts
        rec[key + "__states"] = np.array(S)
        rec[key + "__time_step"] = np.array(env.time_step)
    return rec


def synthetic_value_table():
    """Exactly reproducible fp32 15^6 table: integer bowl + dyadic hash noise (ties included)."""
    i = np.indices((15,) * 6, dtype=np.int64)
    bowl = (i[3] - 7) ** 2 + (i[4] - 7) ** 2 + 2 * (i[5] - 7) ** 2 + (i[0] - 7) - (i[1] - 7)
    lin = np.arange(15 ** 6, dtype=np.uint64).reshape((15,) * 6)
    h = ((lin * np.uint64(2654435761)) >> np.uint64(13)) & np.uint64(255)
    return (bowl.astype(np.float32) + (h.astype(np.float32) - np.float32(128)) / np.float32(64)).astype(np.float32)


def hj_vectors():
    from phoenix_drone_simulation.adversarial_generation.FasTrack_data import distur_gener as dg
    V = synthetic_value_table()
    rec = {}
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as td:
        d = os.path.join(td, "phoenix_drone_simulation/adversarial_generation/FasTrack_data")
        os.makedirs(d)
        levels = [0.0, 1.5, 3.0]
        for lv in levels:
            np.save(os.path.join(d, f"fastrack_{lv}_15x15.npy"), V)
        os.chdir(td)
        try:
            rng = np.random.default_rng(6)
            S = np.concatenate([rng.uniform(-1.6, 1.6, (300, 3)), rng.uniform(-4, 4, (300, 3))], 1)
            g = np.linspace(-math.pi, math.pi, 15)
            S[:60, 3:] = g[rng.integers(0, 15, (60, 3))]                          # exact nodes
            S[60:120, 3:] = (0.5 * (g[:-1] + g[1:]))[rng.integers(0, 14, (60, 3))]  # mid-points (ties)
            S[120:150, 3:] = rng.choice([-math.pi, math.pi, -5.0, 5.0], (30, 3))    # boundary rows
            out = {lv: [] for lv in levels}
            for s in S:
                for lv in levels:
                    u, dd = dg.distur_gener(s, lv)
                    out[lv].append(np.concatenate([np.asarray(u, float).ravel(), np.asarray(dd, float).ravel()]))
        finally:
            os.chdir(cwd)
    rec["states"] = S
    for lv in levels:
        rec[f"ud_{lv}"] = np.array(out[lv])
    return rec


FIXTURES = {"golden_components.npz": lambda: components(),
            "golden_hj.npz": lambda: hj_vectors(),
            "golden_env_trajectories.npz": lambda: env_trajectories(),
            "golden_ground_effect.npz": lambda: ground_effect_trajectories(),
            "golden_env_hj_trajectories.npz": lambda: env_hj_trajectories(),
            "golden_env_uniform_trajectories.npz": lambda: env_uniform_trajectories(),
            "golden_reset_samples.npz": lambda: reset_samples()}


def main(names=None):
    """Write every fixture, or only the ones named on the command line."""
    install_stubs()
    for f in names or FIXTURES:
        np.savez_compressed(os.path.join(HERE, f), **FIXTURES[f]())
        print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main(sys.argv[1:])
