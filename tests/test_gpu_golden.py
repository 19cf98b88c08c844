"""The HIP kernels pinned directly on the reference's fixtures and on analytic known answers.

1. Golden env trajectories (tests/golden/golden_env_trajectories.npz, produced by the reference's
   own Python from its real-flight PWM logs, experiments/07_control_structure_hypothesis/logs/PWM):
   each recorded post-reset state is loaded into the kernel with cf2_set_state and the recorded
   actions are replayed through cf2_step; observations and rewards must match the reference's
   fp64 values to 2e-5 (|g - r| / (1 + |r|); the fp32 restatement is at ~2e-6), dones and costs
   exactly.  The Bullet rigid-body step inside these fixtures is restated by the fixture generator
   (PyBullet is absent): for it the pin is the restatement, not PyBullet.
2. Known answers of the rigid-body step (hover equilibrium, free fall with Bullet damping,
   torque-free rotation invariants, torque / disturbance signs, drag sign), run on the kernel
   through the physics plug-in (cf2_physics_step) from states set with cf2_set_state.
3. Ground effect (tests/golden/golden_ground_effect.npz): the reference's PyBulletPhysics with
   use_ground_effect=True, replayed sub-step by sub-step through the plug-in.
4. HJ-adversary env-steps (tests/golden/golden_env_hj_trajectories.npz): the reference's own
   step() with distur_gener on the synthetic value table, replayed with that table bound; the
   uniform-random-adversary env-steps (golden_env_uniform_trajectories.npz) with the recorded
   dstb_space.sample() torques passed as external disturbances.
"""
import numpy as np
import pytest
import torch

from cf2sim.config import build_config
from test_golden import ENV_IDS, golden_keys, load

pytestmark = pytest.mark.gpu

DET = dict(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0, max_episode_steps=0)


def _golden_state(sf, si, j, g, key, c):
    """Fill env column j of a public snapshot with the reference env's state right after reset()
    (as tests/test_golden.oracle_from_golden does for the restatement)."""
    sf[:, j] = 0.0
    obs0 = g[key + "__obs0"]
    if "Simple" in key:
        sf[0:3, j] = g[key + "__init_xyz"]; sf[3:7, j] = g[key + "__init_quat"]; sf[7:10, j] = g[key + "__init_xyz_dot"]
        sf[10:13, j] = g[key + "__init_rpy_dot"]; sf[13:16, j] = g[key + "__init_rpy"]
    else:
        sf[0:3, j] = g[key + "__init_p"]; sf[3:7, j] = g[key + "__init_q"]; sf[7:10, j] = g[key + "__init_v"]
        sf[10:13, j] = g[key + "__init_w"]
    sf[16:20, j] = g[key + "__init_x"]
    abuf = g[key + "__init_abuf"]
    for r in range(abuf.shape[0]):
        sf[24 + 4 * r:28 + 4 * r, j] = abuf[r]
    sf[56:73, j] = obs0[21:38]
    sf[73:77, j] = obs0[17:21]; sf[77:81, j] = obs0[38:42]
    sf[81, j] = c.time_step; sf[82, j] = c.mass; sf[83:86, j] = (c.ixx, c.iyy, c.izz)
    sf[86, j] = c.ft0; sf[87, j] = c.ft1
    sf[88:92, j] = c.A; sf[92:96, j] = c.B; sf[96:100, j] = c.K
    si[:, j] = 0
    si[2, j] = (1 << 4) | (1 << 5) | (1 << 6)


@pytest.mark.parametrize("family", sorted(ENV_IDS))
def test_kernel_replays_reference_trajectories(gpu, family):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    g = load("golden_env_trajectories.npz")
    keys = [k for k in golden_keys() if k.split("__")[0] == family]
    env_id = ENV_IDS[family]
    n = len(keys)
    kw = dict(DET, auto_reset=False)
    env = BatchedCrazyflieEnv(env_id, n, seed=0, **kw)
    c = build_config(env_id, n, seed=0, **kw)
    sf, si = env.get_state()
    sf, si = sf.cpu().numpy().astype(np.float64), si.cpu().numpy()
    for j, key in enumerate(keys):
        _golden_state(sf, si, j, g, key, c)
    env.set_state(torch.from_numpy(sf.astype(np.float32)), torch.from_numpy(si))
    T = max(len(g[k + "__actions"]) for k in keys)
    worst_o = worst_r = 0.0
    for t in range(T):
        a = np.stack([g[k + "__actions"][min(t, len(g[k + "__actions"]) - 1)] for k in keys]).astype(np.float32)
        o, r, d, info = env.step(torch.from_numpy(a).cuda())
        o, r, d, cost = o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy(), info["cost"].cpu().numpy()
        for j, k in enumerate(keys):
            if t >= len(g[k + "__actions"]):
                continue
            ro = g[k + "__obs"][t]
            worst_o = max(worst_o, float((np.abs(o[j] - ro) / (1 + np.abs(ro))).max()))
            rr = g[k + "__rew"][t]
            worst_r = max(worst_r, abs(float(r[j]) - rr) / (1 + abs(rr)))
            assert bool(d[j]) == bool(g[k + "__done"][t]), (k, t)
            assert cost[j] == g[k + "__cost"][t], (k, t)
    env.close()
    assert worst_o < 2e-5, worst_o
    assert worst_r < 2e-5, worst_r


# ---- known answers of the rigid-body step, on the kernel (through cf2_physics_step) ----

def _drone(cfg):
    from cf2sim.physics import BatchedDrone
    d = BatchedDrone(config=cfg)
    d.reset()
    return d


def _set(drone, p=(0, 0, 1), q=(0, 0, 0, 1), v=(0, 0, 0), w=(0, 0, 0), x=None, abuf=None):
    sf, si = drone.env.get_state()
    sf, si = sf.cpu().numpy(), si.cpu().numpy()
    c = drone.env.cfg
    sf[0:3] = np.asarray(p, np.float32)[:, None]; sf[3:7] = np.asarray(q, np.float32)[:, None]
    sf[7:10] = np.asarray(v, np.float32)[:, None]; sf[10:13] = np.asarray(w, np.float32)[:, None]
    sf[16:20] = np.asarray(x if x is not None else [c.hover_x] * 4, np.float32)[:, None]
    sf[20:24] = 0.0
    sf[24:40] = 0.0
    sf[24:32] = np.asarray(abuf if abuf is not None else [c.hover_action] * 8, np.float32)[:, None]
    sf[104:108] = 0.0
    si[0] = 0; si[2] = 0                    # episode step 0, ring index 0, props at rest
    drone.env.set_state(torch.from_numpy(sf), torch.from_numpy(si))


def _state(drone):
    return drone.env.get_state()[0].cpu().numpy().astype(np.float64)


def _cfg(n=1, **kw):
    base = dict(DET, enable_reset_distribution=False, auto_reset=False)
    base.update(kw)
    return build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", n, seed=1, **base)


def test_kernel_hover_equilibrium(gpu):
    """a = HOVER_ACTION => x -> HOVER_X, and 4 K HOVER_X^2 = m g (agents.py:152-153): 2 s of hover."""
    from cf2sim.physics import PyBulletPhysics
    c = _cfg()
    drone = _drone(c)
    _set(drone)
    phys = PyBulletPhysics(drone, None, time_step=None)
    a = torch.full((1, 4), c.hover_action, device="cuda")
    for _ in range(400):
        phys.step_forward(a)
    s = _state(drone)
    np.testing.assert_allclose(s[16:20, 0] + s[104:108, 0], c.hover_x, rtol=1e-6)
    assert abs(s[9, 0]) < 1e-4 and abs(s[2, 0] - 1.0) < 1e-4
    np.testing.assert_allclose(s[3:7, 0], [0, 0, 0, 1], atol=1e-6)
    drone.close()


def test_kernel_free_fall_with_bullet_damping(gpu):
    """Motors off: v' = -g - 0.04 (1+|v|) v m/m_tot, semi-implicit Euler (fp64 recurrence)."""
    from cf2sim.physics import PyBulletPhysics
    c = _cfg()
    drone = _drone(c)
    _set(drone, p=(0, 0, 10), x=[0] * 4, abuf=[-1.0] * 8)
    phys = PyBulletPhysics(drone, None, time_step=None)
    v, z, dt, mt = 0.0, 10.0, c.time_step, c.mass + 4 * c.prop_mass
    a = torch.full((1, 4), -1.0, device="cuda")
    for _ in range(100):
        phys.step_forward(a)
        v = v + (-9.81 - 0.04 * (1 + abs(v)) * c.mass / mt * v) * dt
        z = z + v * dt
    s = _state(drone)
    assert abs(s[9, 0] - v) < 1e-5 * abs(v) and abs(s[2, 0] - z) < 1e-5 * abs(z)
    assert np.all(s[16:20, 0] == 0.0)
    drone.close()


def test_kernel_torque_free_rotation_invariants(gpu):
    """Damping, gravity and the prop gyrostat off: |L_world| and rotational energy are conserved
    up to the semi-implicit Euler drift, which is first order in dt (10x smaller step: >5x less)."""
    from cf2sim.physics import PyBulletPhysics
    c = _cfg()
    c.ang_damping = 0.0; c.lin_damping = 0.0; c.prop_inertia = 0.0; c.prop_mass = 0.0; c.gravity_world = 0.0
    I = np.array([c.ixx, c.iyy, c.izz])

    def rot(q):
        x, y, z, w = q
        return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                         [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                         [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])

    def inv(s):
        R = rot(s[3:7, 0]); wb = R.T @ s[10:13, 0]
        return np.linalg.norm(R @ (I * wb)), 0.5 * np.sum(I * wb * wb)

    drift = []
    for scale in (1, 10):
        drone = _drone(c)
        _set(drone, w=(3.0, 0.5, 2.0), x=[0] * 4, abuf=[-1.0] * 8)
        L0, E0 = inv(_state(drone))
        phys = PyBulletPhysics(drone, None, time_step=0.005 / scale, gravity=0.0)
        a = torch.full((1, 4), -1.0, device="cuda")
        for _ in range(200 * scale):
            phys.step_forward(a)
        L1, E1 = inv(_state(drone))
        drift.append(max(abs(L1 - L0) / L0, abs(E1 - E0) / E0))
        drone.close()
    assert drift[0] < 3e-2 and drift[1] < drift[0] / 5, drift


def test_kernel_torque_and_disturbance_signs(gpu):
    """+x / +y adversary torque -> +roll / +pitch rate only (applied on link 4 in its frame,
    physics.py:228-229); motors 1 and 3 faster -> +yaw rate (tz = -t0 + t1 - t2 + t3)."""
    from cf2sim.physics import PybulletPhysicsWithAdversary
    c = _cfg(n=3)
    c.prop_inertia = 0.0
    drone = _drone(c)
    _set(drone)
    sf, si = drone.env.get_state()
    sf[16:20, 2] = torch.tensor([0.7, 0.8, 0.7, 0.8])
    drone.env.set_state(sf, si)
    phys = PybulletPhysicsWithAdversary(drone, None, time_step=None)
    d = torch.tensor([[1e-3, 0, 0], [0, 1e-3, 0], [0, 0, 0]], device="cuda")
    phys.step_forward(torch.full((3, 4), c.hover_action, device="cuda"), d)
    rd = drone.rpy_dot.cpu().numpy()
    assert rd[0, 0] > 0 and abs(rd[0, 1]) < 1e-6
    assert rd[1, 1] > 0 and abs(rd[1, 0]) < 1e-6
    assert rd[2, 2] > 0
    drone.close()


def test_kernel_drag_opposes_velocity(gpu):
    from cf2sim.physics import PyBulletPhysics
    vx = []
    for drag in (None, 0.0):
        c = _cfg()
        if drag is not None:
            c.drag_xy = drag
        drone = _drone(c)
        _set(drone, p=(0, 0, 5), v=(2.0, 0, 0), x=[1.0] * 4, abuf=[1.0] * 8)
        PyBulletPhysics(drone, None, time_step=None).step_forward(torch.ones(1, 4, device="cuda"))
        vx.append(float(_state(drone)[7, 0]))
        drone.close()
    assert vx[0] < vx[1]


def test_kernel_ground_effect_replays_reference(gpu):
    """PyBulletPhysics(use_ground_effect=True) on the kernel (cf2_set_ground_effect +
    cf2_physics_step) replays the reference's ground-effect sub-steps
    (tests/golden/golden_ground_effect.npz, physics.py:27-58, 91-124): p, q, v, w and the motor
    state within 2e-5 of the fp64 reference over 120 sub-steps near the ground, one env per case
    (ge__3 flipped past |roll| = pi/2, where the reference applies none)."""
    from cf2sim.physics import PyBulletPhysics
    from test_golden import ge_keys
    g = load("golden_ground_effect.npz")
    keys = ge_keys()
    n = len(keys)
    c = _cfg(n=n)
    drone = _drone(c)
    sf, si = drone.env.get_state()
    sf, si = sf.cpu().numpy().astype(np.float64), si.cpu().numpy()
    for j, key in enumerate(keys):
        sf[:, j] = 0.0
        sf[0:3, j] = g[key + "__init_p"]; sf[3:7, j] = g[key + "__init_q"]; sf[7:10, j] = g[key + "__init_v"]
        sf[10:13, j] = g[key + "__init_w"]; sf[16:20, j] = g[key + "__init_x"]
        abuf = g[key + "__init_abuf"]
        for r in range(abuf.shape[0]):
            sf[24 + 4 * r:28 + 4 * r, j] = abuf[r]
        sf[81, j] = c.time_step; sf[82, j] = c.mass; sf[83:86, j] = (c.ixx, c.iyy, c.izz)
        sf[86, j] = c.ft0; sf[87, j] = c.ft1
        sf[88:92, j] = c.A; sf[92:96, j] = c.B; sf[96:100, j] = c.K
        si[:, j] = 0
    drone.env.set_state(torch.from_numpy(sf.astype(np.float32)), torch.from_numpy(si))
    phys = PyBulletPhysics(drone, None, time_step=None, use_ground_effect=True)
    acts = np.stack([g[k + "__actions"] for k in keys], 1)          # (T, n, 4)
    worst = 0.0
    for t in range(acts.shape[0]):
        phys.step_forward(torch.from_numpy(np.ascontiguousarray(acts[t])).cuda())
        s = _state(drone)
        for j, k in enumerate(keys):
            got = np.concatenate([s[0:13, j], s[16:20, j] + s[104:108, j]])
            ref = g[k + "__states"][t]
            worst = max(worst, float((np.abs(got - ref) / (1 + np.abs(ref))).max()))
    drone.close()
    assert worst < 2e-5, worst


@pytest.mark.parametrize("family", ["DroneHoverBulletFreeEnvWithAdversary", "DroneHoverBulletEnvWithAdversary",
                                    "DroneHoverBulletFreeEnvWithRandomHJAdversary"])
def test_kernel_replays_reference_hj_trajectories(gpu, family):
    """The HJ-adversary env-steps of the reference (tests/golden/golden_env_hj_trajectories.npz:
    distur_gener on the synthetic value table inside the reference's own step()) replayed on the
    kernel with the same table bound: obs and reward within 2e-5 of the fp64 reference, done and
    cost exact (the nearest-node search and the sign rule are exact; only fp32 rounding of the
    state differs)."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    from test_golden import HJ_ENV_IDS, hj_golden_keys, synthetic_value_table
    g = load("golden_env_hj_trajectories.npz")
    keys = [k for k in hj_golden_keys() if k.split("__")[0] == family]
    env_id, n = HJ_ENV_IDS[family], len(keys)
    kw = dict(DET, auto_reset=False)
    if "Random" not in family:
        kw["disturbance_level"] = float(g[keys[0] + "__level"])
    env = BatchedCrazyflieEnv(env_id, n, seed=0, **kw)
    c = build_config(env_id, n, seed=0, **kw)
    env.bind_hj_tables(torch.from_numpy(synthetic_value_table()).reshape(1, -1).cuda(), [0] * int(c.num_levels))
    sf, si = env.get_state()
    sf, si = sf.cpu().numpy().astype(np.float64), si.cpu().numpy()
    for j, key in enumerate(keys):
        _golden_state(sf, si, j, g, key, c)
        sf[103, j] = g[key + "__level"]
    env.set_state(torch.from_numpy(sf.astype(np.float32)), torch.from_numpy(si))
    T = max(len(g[k + "__actions"]) for k in keys)
    worst_o = worst_r = 0.0
    for t in range(T):
        a = np.stack([g[k + "__actions"][min(t, len(g[k + "__actions"]) - 1)] for k in keys]).astype(np.float32)
        o, r, d, info = env.step(torch.from_numpy(a).cuda())
        o, r, d, cost = o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy(), info["cost"].cpu().numpy()
        for j, k in enumerate(keys):
            if t >= len(g[k + "__actions"]):
                continue
            ro = g[k + "__obs"][t]
            worst_o = max(worst_o, float((np.abs(o[j] - ro) / (1 + np.abs(ro))).max()))
            rr = g[k + "__rew"][t]
            worst_r = max(worst_r, abs(float(r[j]) - rr) / (1 + abs(rr)))
            assert bool(d[j]) == bool(g[k + "__done"][t]), (k, t)
            assert cost[j] == g[k + "__cost"][t], (k, t)
    env.close()
    assert worst_o < 2e-5, worst_o
    assert worst_r < 2e-5, worst_r


@pytest.mark.parametrize("family", ["DroneHoverBulletFreeEnvWithRandomAdversary", "DroneHoverBulletEnvWithRandomAdversary"])
def test_kernel_replays_reference_uniform_adversary_trajectories(gpu, family):
    """The uniform-random-adversary env-steps of the reference
    (tests/golden/golden_env_uniform_trajectories.npz) replayed on the kernel with each step's
    recorded dstb_space.sample() passed as the external disturbance (cf2_step's dstb_dev): obs and
    reward within 2e-5 of the fp64 reference, done and cost exact."""
    from cf2sim.config import DSTB_EXTERNAL
    from cf2sim.vec_env import BatchedCrazyflieEnv
    from test_golden import UNI_ENV_IDS, uniform_golden_keys
    g = load("golden_env_uniform_trajectories.npz")
    keys = [k for k in uniform_golden_keys() if k.split("__")[0] == family]
    env_id, n = UNI_ENV_IDS[family], len(keys)
    kw = dict(DET, auto_reset=False, disturbance=DSTB_EXTERNAL)
    env = BatchedCrazyflieEnv(env_id, n, seed=0, **kw)
    c = build_config(env_id, n, seed=0, **kw)
    sf, si = env.get_state()
    sf, si = sf.cpu().numpy().astype(np.float64), si.cpu().numpy()
    for j, key in enumerate(keys):
        _golden_state(sf, si, j, g, key, c)
    env.set_state(torch.from_numpy(sf.astype(np.float32)), torch.from_numpy(si))
    T = max(len(g[k + "__actions"]) for k in keys)
    worst_o = worst_r = 0.0
    for t in range(T):
        a = np.stack([g[k + "__actions"][min(t, len(g[k + "__actions"]) - 1)] for k in keys]).astype(np.float32)
        dv = np.stack([g[k + "__dstb"][min(t, len(g[k + "__dstb"]) - 1)] for k in keys]).astype(np.float32)
        o, r, d, info = env.step(torch.from_numpy(a).cuda(), torch.from_numpy(dv).cuda())
        o, r, d, cost = o.cpu().numpy(), r.cpu().numpy(), d.cpu().numpy(), info["cost"].cpu().numpy()
        for j, k in enumerate(keys):
            if t >= len(g[k + "__actions"]):
                continue
            ro = g[k + "__obs"][t]
            worst_o = max(worst_o, float((np.abs(o[j] - ro) / (1 + np.abs(ro))).max()))
            rr = g[k + "__rew"][t]
            worst_r = max(worst_r, abs(float(r[j]) - rr) / (1 + abs(rr)))
            assert bool(d[j]) == bool(g[k + "__done"][t]), (k, t)
            assert cost[j] == g[k + "__cost"][t], (k, t)
    env.close()
    assert worst_o < 2e-5, worst_o
    assert worst_r < 2e-5, worst_r


@pytest.mark.parametrize("key", ["samples_hover", "samples_initial", "samples_randomhj"])
def test_kernel_reset_distribution_other_classes(gpu, key):
    """cf2_reset of the hover, AdversaryInitial and Boltzmann-level env classes at 65 536 envs vs
    the reference's reset() samples of the same class (KS per field, chi-square on the level)."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    from test_golden import RESET_CASES, reset_ks_pvalues
    env = BatchedCrazyflieEnv(RESET_CASES[key], 65536, seed=31)
    env.reset()
    sf = env.get_state()[0].cpu().numpy().astype(np.float64)
    env.close()
    p = reset_ks_pvalues(sf, key)
    bad = {k: v for k, v in p.items() if v < 1e-4}
    assert not bad, bad


def test_kernel_reset_distribution_matches_reference_samples(gpu):
    """The kernel's reset (cf2_reset at 65 536 envs, and the in-step auto-resets of a second batch
    after 60 random-action env-steps) vs the reference's own reset() samples
    (tests/golden/golden_reset_samples.npz): every pose / velocity / motor / action-ring / DR field
    and the sampled body rates R(q) w are one distribution by a two-sample KS test (p > 1e-4)."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    from test_golden import reset_ks_pvalues
    env_id = "DroneHoverBulletFreeEnvWithoutAdversary-v0"
    env = BatchedCrazyflieEnv(env_id, 65536, seed=23)
    env.reset()
    sf = env.get_state()[0].cpu().numpy().astype(np.float64)
    env.close()
    p = reset_ks_pvalues(sf)
    bad = {k: v for k, v in p.items() if v < 1e-4}
    assert not bad, bad
    # auto-resets inside the step kernel (role-split block epilogue): collect the state of envs
    # right after their reset (episode step 0 after a done)
    env = BatchedCrazyflieEnv(env_id, 65536, seed=29)
    env.reset()
    gen = torch.Generator(device="cuda")
    gen.manual_seed(4)
    rows = []
    for t in range(60):
        _, _, d, _ = env.step((torch.rand(65536, 4, device="cuda", generator=gen) * 2 - 1).contiguous())
        if t % 6 == 5:
            sf, si = env.get_state()
            fresh = (si[0] == 0).cpu().numpy()
            rows.append(sf.cpu().numpy().astype(np.float64)[:, fresh])
    env.close()
    sf = np.concatenate(rows, 1)
    assert sf.shape[1] > 3000, sf.shape
    p = reset_ks_pvalues(sf)
    bad = {k: v for k, v in p.items() if v < 1e-4}
    assert not bad, bad
