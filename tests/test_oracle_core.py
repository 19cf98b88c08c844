"""CPU tests of the restatement (oracle/): known answers, invariants and analytic solutions.

The reference holds no numeric test of its dynamics; these checks pin
the restatement on analytic ground truth, and tests/test_golden.py pins it on vectors
produced by the reference's own Python.
"""
import math

import numpy as np
import pytest

import oracle as O
from cf2sim.config import build_config


def cfg_det(env_id="DroneHoverBulletFreeEnvWithoutAdversary-v0", n=1, **kw):
    base = dict(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0, enable_reset_distribution=False)
    base.update(kw)
    return build_config(env_id, n, seed=1, **base)


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert O.philox([0, 0, 0, 0], [0, 0]) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert O.philox([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6, 0x6d5451fd]
    assert O.philox([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0]) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]
    for prec in ("f32",):
        assert O.philox([1, 2, 3, 4], [5, 6], prec) == O.philox([1, 2, 3, 4], [5, 6])


def test_quaternion_round_trip():
    """tests/test_quaternion.py:35-43 of the reference: rpy -> quat -> rpy is the identity."""
    rng = np.random.default_rng(0)
    for _ in range(200):
        rpy = rng.uniform(-1.5, 1.5, 3)
        q = O.quat_from_euler(rpy)
        assert abs(np.linalg.norm(q) - 1) < 1e-14
        np.testing.assert_allclose(O.euler_from_quat(q), rpy, atol=1e-12)
        np.testing.assert_allclose(O.quat2euler(q), rpy, atol=1e-12)


def test_rotmat_orthonormal_and_axis():
    rng = np.random.default_rng(1)
    for _ in range(50):
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        R = O.rotmat(q)
        np.testing.assert_allclose(R @ R.T, np.eye(3), atol=1e-13)
        assert abs(np.linalg.det(R) - 1) < 1e-13
    R = O.rotmat(O.quat_from_euler([0.0, 0.0, math.pi / 2]))
    np.testing.assert_allclose(R @ [1, 0, 0], [0, 1, 0], atol=1e-15)


def test_hover_equilibrium_known_answer():
    """a = HOVER_ACTION => x -> HOVER_X and 4 K HOVER_X^2 = m g (agents.py:152-153)."""
    c = cfg_det()
    assert abs(4 * c.K * c.hover_x ** 2 - c.mass * 9.81) < 1e-15
    st = np.zeros(29)
    st[2] = 1.0; st[6] = 1.0
    st[13:17] = c.hover_x
    st[21:29] = c.hover_action
    for k in range(400):
        st, _ = O.bullet_substep(c, st, [c.hover_action] * 4, [0, 0, 0], [0] * 4, first_after_reset=(k == 0))
    np.testing.assert_allclose(st[13:17], c.hover_x, rtol=1e-12)
    # vz ~ 0, z ~ 1 after 2 s; the 4 x 1e-9 kg props make gravity exceed thrust by 1.3e-7 relative
    assert abs(st[9]) < 1e-5 and abs(st[2] - 1.0) < 1e-5
    np.testing.assert_allclose(st[3:7], [0, 0, 0, 1], atol=1e-12)


def test_free_fall_with_bullet_damping():
    """Motors off: v' = -g m_tot/m_tot - 0.04 (1+|v|) v m/m_tot, semi-implicit Euler."""
    c = cfg_det(motor_thrust_noise=0)
    st = np.zeros(29); st[2] = 10.0; st[6] = 1.0
    st[21:29] = -1.0
    v, z = 0.0, 10.0
    dt = c.time_step
    mt = c.mass + 4 * c.prop_mass
    for k in range(100):
        st, _ = O.bullet_substep(c, st, [-1.0] * 4, [0, 0, 0], [0] * 4, first_after_reset=(k == 0))
        acc = -9.81 - 0.04 * (1 + abs(v)) * c.mass / mt * v
        v = v + acc * dt
        z = z + v * dt
    assert abs(st[9] - v) < 1e-12 and abs(st[2] - z) < 1e-12
    assert np.all(st[13:17] == 0.0)


def test_torque_free_rotation_conserves_energy_and_momentum():
    """Pure gyroscopic motion (damping off): |L_world| and rotational energy are conserved to
    O(dt) per step; checks the w x Iw sign and the exp-map integration."""
    c = cfg_det()
    c.ang_damping = 0.0; c.lin_damping = 0.0; c.prop_inertia = 0.0; c.prop_mass = 0.0; c.gravity_world = 0.0
    st = np.zeros(29); st[6] = 1.0
    st[10:13] = [3.0, 0.5, 2.0]      # world angular velocity
    I = np.array([c.ixx, c.iyy, c.izz])
    def invariants(s):
        R = O.rotmat(s[3:7]); wb = R.T @ s[10:13]
        return np.linalg.norm(R @ (I * wb)), 0.5 * np.sum(I * wb * wb)
    L0, E0 = invariants(st)
    drift = []
    for scale in (1, 10):      # semi-implicit Euler: drift is first order in dt
        s = st.copy()
        c.time_step = 0.005 / scale
        for k in range(200 * scale):
            s, _ = O.bullet_substep(c, s, [-1.0] * 4, [0, 0, 0], [0] * 4, True)
        L1, E1 = invariants(s)
        drift.append(max(abs(L1 - L0) / L0, abs(E1 - E0) / E0))
    assert drift[0] < 3e-2 and drift[1] < drift[0] / 5, drift


def test_pure_yaw_torque_and_roll_disturbance_signs():
    c = cfg_det()
    c.prop_inertia = 0.0
    base = np.zeros(29); base[2] = 1.0; base[6] = 1.0
    base[13:17] = c.hover_x; base[21:29] = c.hover_action
    # positive x-torque disturbance -> positive roll rate (applied on link 4 in its frame)
    st, rw = O.bullet_substep(c, base.copy(), [c.hover_action] * 4, [1e-3, 0, 0], [0] * 4)
    assert rw[3] > 0 and abs(rw[4]) < 1e-12
    st, rw = O.bullet_substep(c, base.copy(), [c.hover_action] * 4, [0, 1e-3, 0], [0] * 4)
    assert rw[4] > 0 and abs(rw[3]) < 1e-12
    # motors 1 and 3 (indices 1,3) faster -> positive yaw torque tz = -t0 + t1 - t2 + t3
    b2 = base.copy(); b2[13:17] = [0.7, 0.8, 0.7, 0.8]
    st, rw = O.bullet_substep(c, b2, [c.hover_action] * 4, [0, 0, 0], [0] * 4)
    assert rw[5] > 0


def test_drag_opposes_velocity():
    c = cfg_det()
    st = np.zeros(29); st[2] = 5.0; st[6] = 1.0; st[7] = 2.0   # vx = 2 m/s, level attitude
    st[13:17] = 1.0; st[21:29] = 1.0
    s1, _ = O.bullet_substep(c, st.copy(), [1.0] * 4, [0, 0, 0], [0] * 4)
    c2 = cfg_det(); c2.drag_xy = 0.0
    s2, _ = O.bullet_substep(c2, st.copy(), [1.0] * 4, [0, 0, 0], [0] * 4)
    assert s1[7] < s2[7]


def test_reset_distribution_bounds_and_quirks():
    c = build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", 4000, seed=5, observation_noise=0)
    env = O.OracleEnv(c)
    env.reset()
    sf, si = env.get_state()
    pos, vel = sf[0:3], sf[7:10]
    assert np.all(np.abs(pos - np.array([[0], [0], [1]])) <= 0.25)
    assert np.all(np.abs(vel) <= 0.1)
    x = sf[16:20]
    assert abs(x.mean() - c.hover_x) < 2e-3 and abs(x.std() - 0.02) < 2e-3
    abuf = sf[24:32]
    assert np.all(np.abs(abuf) <= 1) and abs(abuf.mean() - c.hover_action) < 2e-3
    dt = sf[81]
    assert np.all((dt >= 0.005 * 0.9 - 1e-12) & (dt <= 0.005 * 1.1 + 1e-12))
    # DR K uses 0.028 kg (agents.py:224), not M = 0.030
    K = sf[96:100]
    assert K.max() <= 0.028 * 9.81 * 1.8 * 1.1 / 4 + 1e-12
    # alias bits set after reset (both action_history entries view action_buffer[-1])
    assert np.all((si[2] >> 4) & 3 == 3)
    env.close()


def test_history_alias_quirk():
    """base.py:455-460 appends the *view* drone.last_action = action_buffer[-1]; the first two
    histories therefore show the buffer row that apply_action overwrote."""
    c = build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", 1, seed=2, observation_noise=0,
                     domain_randomization=-1, motor_thrust_noise=0)
    env = O.OracleEnv(c)
    o0 = env.reset()
    a1 = np.full((1, 4), 0.3, np.float32); a2 = np.full((1, 4), -0.2, np.float32); a3 = np.full((1, 4), 0.05, np.float32)
    o1, *_ = env.step(a1)
    o2, *_ = env.step(a2)
    o3, *_ = env.step(a3)
    A = lambda o, k: o[0, 17:21] if k == 0 else o[0, 38:42]
    np.testing.assert_allclose(A(o1, 0), 0.3, atol=1e-7); np.testing.assert_allclose(A(o1, 1), 0.3, atol=1e-7)
    np.testing.assert_allclose(A(o2, 0), -0.2, atol=1e-7); np.testing.assert_allclose(A(o2, 1), 0.3, atol=1e-7)
    np.testing.assert_allclose(A(o3, 0), 0.3, atol=1e-7); np.testing.assert_allclose(A(o3, 1), -0.2, atol=1e-7)
    # obs17 = state17 carries last_action = current action
    np.testing.assert_allclose(o3[0, 34:38], 0.05, atol=1e-7)
    env.close()


def test_time_limit_truncation_and_auto_reset():
    c = cfg_det(max_episode_steps=5)
    env = O.OracleEnv(c)
    env.reset()
    for k in range(5):
        o, r, d, info = env.step(np.full((1, 4), c.hover_action, np.float32))
    assert d[0] and info["truncated"][0]
    sf, si = env.get_state()
    assert si[0, 0] == 0          # auto-reset happened
    env.close()


def test_boltzmann_distribution_matches_reference_probabilities():
    from cf2sim.config import boltzmann_table
    c = build_config("DroneHoverBulletFreeEnvWithRandomHJAdversary-v0", 1)
    values, cdf = boltzmann_table()
    assert len(values) == 21 and values[0] == 0.0 and values[-1] == 2.0
    us = (np.arange(1 << 14) + 0.5) / (1 << 14)
    idx = np.array([O.boltzmann_index(c, u) for u in us])
    ref = np.searchsorted(cdf, us, side="right")
    np.testing.assert_array_equal(idx, ref)


def test_reward_done_cost_known_answers():
    c = build_config("DroneHoverBulletFreeEnvWithAdversary-v0", 1)
    attrs = np.zeros(16); attrs[2] = 1.0
    r, d, cost = O.reward_done_cost(c, attrs, [0.1] * 4)
    assert r == 0.0 and not d and cost == 0.0
    attrs[3:6] = [0.3, -0.4, 0.0]            # |rpy| = 0.5 rad, roll > 10 deg -> cost
    attrs[9:12] = [0.0, 0.0, 2.0]
    attrs[6:9] = [0.0, 0.3, 0.4]
    r, d, cost = O.reward_done_cost(c, attrs, [0.1] * 4)
    assert abs(r - -(0.5 + 2.0 + 0.5)) < 1e-12 and not d and cost == 1.0
    attrs[3] = np.deg2rad(76.0)               # > 75 deg -> done, terminal penalty 1000
    r, d, _ = O.reward_done_cost(c, attrs, [0.1] * 4)
    assert d and r < -1000
    attrs = np.zeros(16); attrs[2] = 0.19
    assert O.reward_done_cost(c, attrs, [0.1] * 4)[1]
    attrs = np.zeros(16); attrs[2] = 1.0; attrs[11] = np.deg2rad(1001)
    assert O.reward_done_cost(c, attrs, [0.1] * 4)[1]
    hov = build_config("DroneHoverBulletEnv-v0", 1)    # 60 deg / 300 deg/s and the -dist term
    attrs = np.zeros(16); attrs[2] = 1.0; attrs[9] = np.deg2rad(301)
    assert O.reward_done_cost(hov, attrs, [0.1] * 4)[1]
    attrs = np.zeros(16); attrs[0:3] = [0.3, 0.0, 1.4]
    r, d, _ = O.reward_done_cost(hov, attrs, [1.0] * 4)
    assert abs(r - -(0.5 + 1e-4 * 2.0)) < 1e-12


@pytest.mark.parametrize("env_id,kw", [("DroneHoverBulletFreeEnvWithGust-v0", {}),
                                        ("DroneHoverBulletFreeEnvWithDownwash-v0", {"num_drones": 4})])
def test_threaded_step_is_bit_identical(env_id, kw):
    """The all-core CPU baseline (bench.py) steps formations on OpenMP threads: same results."""
    c = build_config(env_id, 256, seed=5, **kw)
    e1 = O.OracleEnv(c, "f64"); e4 = O.OracleEnv(c, "f64")
    e4.set_threads(4)
    np.testing.assert_array_equal(e1.reset(), e4.reset())
    rng = np.random.default_rng(2)
    for t in range(40):
        a = rng.uniform(-1, 1, (256, 4)).astype(np.float32)
        r1, r4 = e1.step(a, want_final=True), e4.step(a, want_final=True)
        for x, y in zip(r1[:3], r4[:3]):
            np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(r1[3]["final_obs"], r4[3]["final_obs"])
    s1, s4 = e1.get_state(), e4.get_state()
    np.testing.assert_array_equal(s1[0], s4[0]); np.testing.assert_array_equal(s1[1], s4[1])
    e1.close(); e4.close()


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_fp32_restatement_tracks_fp64(prec):
    c = build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", 64, seed=9)
    e64 = O.OracleEnv(c, "f64"); ex = O.OracleEnv(c, prec)
    o64 = e64.reset(); ox = ex.reset()
    rng = np.random.default_rng(3)
    for t in range(60):
        a = (rng.uniform(-1, 1, (64, 4)) * 0.2 + 0.111).astype(np.float32)
        o64, r64, d64, _ = e64.step(a)
        ox, rx, dx, _ = ex.step(a)
    assert np.abs(o64 - ox).max() < (1e-12 if prec == "f64" else 2e-3)


@pytest.mark.parametrize("noisy", [False, True])
def test_fp32_restatement_meets_state_tolerance(noisy):
    """The fp32 restatement (the kernel's arithmetic, incl. the compensated motor state) tracks the
    fp64 restatement within BASELINE.json's 1e-4 state tolerance over 240 closed-loop env-steps
    (metric: parity_util.state_rel_err).  The GPU tests hold the kernel to the same bound."""
    from parity_util import CLEAN, pd_actions, state_rel_err
    env_id = "DroneHoverBulletFreeEnvWithoutAdversary-v0"
    kw = dict(max_episode_steps=0) if noisy else CLEAN
    n = 128
    sl = slice(17, 30) if noisy else slice(21, 34)
    a32 = O.OracleEnv(build_config(env_id, n, seed=11, **kw), "f32")
    a64 = O.OracleEnv(build_config(env_id, n, seed=11, **kw), "f64")
    cfg = a64.cfg
    go, ro = a32.reset(), a64.reset()
    for _ in range(240):
        go = a32.step(pd_actions(go[:, sl], cfg.hover_action))[0]
        ro = a64.step(pd_actions(ro[:, sl], cfg.hover_action))[0]
    g, r = a32.get_state()[0][:13], a64.get_state()[0][:13]
    worst = {k: float(v.max()) for k, v in state_rel_err(g, r).items()}
    assert max(worst.values()) < 1e-4, worst
