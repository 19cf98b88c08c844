"""Pin the CPU restatement (oracle/) on golden vectors produced by running the REFERENCE's own
Python (tests/golden/make_golden.py; fixtures are data, the reference is not read here).

What each fixture pins (reference file:line):
* aa_*   CrazyFlieAgent.apply_action + PWM.act + OUNoise (agents.py:259-298, control.py:94-100,
         utils.py:111-134), OU draws recorded
* sn_*   SensorNoise.add_noise / add_noise_to_omega (sensors.py:75-134), draws recorded
* q_*    get_quaternion_from_euler (utils.py:58-82), quat2euler (distur_gener.py:186-207)
* boltz  Boltzmann() probabilities (utils.py:27-39)
* hj     distur_gener() incl. Grid.get_index and the boundary rules (distur_gener.py:19-183,
         GridProcessing.py:52-71) on an exactly reproducible synthetic value table
* env_hj whole env-steps of the HJ-adversary envs (fixed level: hover_free and hover; Boltzmann
         level) on the synthetic value table, distur_gener run by the reference's step()
* env    whole env-steps of DroneHoverBulletFreeEnvWithoutAdversary / DroneHoverBulletEnv /
         DroneHoverBulletEnvWithoutAdversary / DroneHoverSimpleEnv driven by the reference's
         real-flight PWM logs: apply_action, latency ring, drag, force/torque assembly,
         update_information, compute_observation/history (with the action-buffer alias),
         reward/done/info are the reference's code; SimplePhysics is the reference's code; the
         Bullet integrator inside the fake physics server is a numpy restatement (PyBullet is
         not installable here: parity of that one piece vs PyBullet is unpinned).
* ge     PyBulletPhysics(use_ground_effect=True).step_forward near the ground: calculate_ground_effect
         (physics.py:27-58) with the prop heights from getLinkStates, every sub-step recorded
"""
import os

import numpy as np
import pytest

import oracle as O
from cf2sim.config import boltzmann_table, build_config

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(GOLD, name), allow_pickle=False)


def test_apply_action_matches_reference():
    g = load("golden_components.npz")
    c = build_config("DroneHoverBulletEnv-v0", 1)
    f, tz, x = O.apply_action(c, g["aa_actions"], g["aa_ou_normals"], g["aa_init_x"], g["aa_init_buf"])
    np.testing.assert_allclose(f, g["aa_forces"], rtol=1e-13, atol=1e-16)
    np.testing.assert_allclose(tz, g["aa_tz"], rtol=1e-12, atol=1e-16)
    np.testing.assert_allclose(x, g["aa_x"], rtol=1e-14)


def test_sensor_noise_matches_reference():
    g = load("golden_components.npz")
    c = build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", 1)
    ins, draws, outs = g["sn_in"], g["sn_draws"], g["sn_out"]
    for k in range(len(ins)):
        pos, vel, rot, om, bias = ins[k][0:3], ins[k][3:6], ins[k][6:9], ins[k][9:12], ins[k][12:15]
        p, v, r, o, b = O.add_noise(c, pos, vel, rot, om, draws[k][:18], draws[k][18:24], bias)
        np.testing.assert_allclose(np.concatenate([p, v, r, o, b]), outs[k], rtol=1e-14, atol=1e-15)


def test_quaternion_conversions_match_reference():
    g = load("golden_components.npz")
    for rpy, q in zip(g["q_rpy"], g["q_utils"]):
        np.testing.assert_allclose(O.quat_from_euler(rpy), q / np.linalg.norm(q), atol=1e-15)
    for q, e in zip(g["q_quats"], g["q_quat2euler"]):
        np.testing.assert_allclose(O.quat2euler(q), e, atol=1e-14)


def test_boltzmann_probabilities_match_reference():
    g = load("golden_components.npz")
    values, cdf = boltzmann_table()
    np.testing.assert_allclose(values, np.around(g["boltz_energies"], 1))
    p = g["boltz_p"]
    np.testing.assert_allclose(np.diff(np.concatenate([[0.0], cdf])), p / p.sum(), rtol=1e-12)


def synthetic_value_table():
    i = np.indices((15,) * 6, dtype=np.int64)
    bowl = (i[3] - 7) ** 2 + (i[4] - 7) ** 2 + 2 * (i[5] - 7) ** 2 + (i[0] - 7) - (i[1] - 7)
    lin = np.arange(15 ** 6, dtype=np.uint64).reshape((15,) * 6)
    h = ((lin * np.uint64(2654435761)) >> np.uint64(13)) & np.uint64(255)
    return (bowl.astype(np.float32) + (h.astype(np.float32) - np.float32(128)) / np.float32(64)).astype(np.float32)


@pytest.fixture(scope="module")
def V():
    return synthetic_value_table()


@pytest.mark.parametrize("level", [0.0, 1.5, 3.0])
def test_hj_disturbance_matches_reference(V, level):
    g = load("golden_hj.npz")
    c = build_config("DroneHoverBulletFreeEnvWithAdversary-v0", 1)
    d, u, idx = O.hj(c, V, g["states"], level)
    ref = g[f"ud_{level}"]
    np.testing.assert_array_equal(u, ref[:, :3])
    np.testing.assert_array_equal(d, ref[:, 3:])


ENV_IDS = {"DroneHoverBulletFreeEnvWithoutAdversary": "DroneHoverBulletFreeEnvWithoutAdversary-v0",
           "DroneHoverBulletEnv": "DroneHoverBulletEnv-v0",
           "DroneHoverBulletEnvWithoutAdversary": "DroneHoverBulletEnvWithoutAdversary-v0",
           "DroneHoverSimpleEnv": "DroneHoverSimpleEnv-v0"}


def oracle_from_golden(g, key, env_id, precision="f64", V=None, **kw):
    """Oracle env whose state is the reference env's state right after its reset() (HJ envs: the
    recorded level, every level on the table V)."""
    c = build_config(env_id, 1, observation_noise=0, domain_randomization=-1, motor_thrust_noise=0,
                     max_episode_steps=0, auto_reset=False, **kw)
    env = O.OracleEnv(c, precision)
    if V is not None:
        env.bind_tables(V, [0] * int(c.num_levels))
    sf, si = env.get_state()
    sf[:] = 0
    simple = "Simple" in key
    obs0 = g[key + "__obs0"]
    if simple:
        sf[0:3, 0] = g[key + "__init_xyz"]; sf[3:7, 0] = g[key + "__init_quat"]; sf[7:10, 0] = g[key + "__init_xyz_dot"]
        sf[10:13, 0] = g[key + "__init_rpy_dot"]; sf[13:16, 0] = g[key + "__init_rpy"]
    else:
        sf[0:3, 0] = g[key + "__init_p"]; sf[3:7, 0] = g[key + "__init_q"]; sf[7:10, 0] = g[key + "__init_v"]
        sf[10:13, 0] = g[key + "__init_w"]
    sf[16:20, 0] = g[key + "__init_x"]
    abuf = g[key + "__init_abuf"]
    for r in range(abuf.shape[0]):
        sf[24 + 4 * r:28 + 4 * r, 0] = abuf[r]
    sf[56:73, 0] = obs0[21:38]                       # o_0 of the reset history
    sf[73:77, 0] = obs0[17:21]; sf[77:81, 0] = obs0[38:42]
    sf[81, 0] = c.time_step; sf[82, 0] = c.mass; sf[83:86, 0] = (c.ixx, c.iyy, c.izz)
    sf[86, 0] = c.ft0; sf[87, 0] = c.ft1
    sf[88:92, 0] = c.A; sf[92:96, 0] = c.B; sf[96:100, 0] = c.K
    if key + "__level" in g.files:
        sf[103, 0] = g[key + "__level"]
    si[:] = 0
    si[2, 0] = (1 << 4) | (1 << 5) | (1 << 6)      # both history entries alias action_buffer[-1]
    env.set_state(sf, si)
    return env


def golden_keys():
    g = load("golden_env_trajectories.npz")
    return sorted({k.split("__")[0] + "__" + k.split("__")[1] for k in g.files})


@pytest.mark.parametrize("key", golden_keys())
def test_env_steps_match_reference(key):
    g = load("golden_env_trajectories.npz")
    env = oracle_from_golden(g, key, ENV_IDS[key.split("__")[0]])
    acts, obs, rew, done, cost = (g[key + s] for s in ("__actions", "__obs", "__rew", "__done", "__cost"))
    assert len(acts) >= 10
    for t in range(len(acts)):
        o, r, d, info = env.step(acts[t:t + 1])
        err = np.abs(o[0] - obs[t]) / (1 + np.abs(obs[t]))
        assert err.max() < 1e-9, (t, err.max(), np.argmax(err))
        assert abs(r[0] - rew[t]) <= 1e-9 * (1 + abs(rew[t])), (t, r[0], rew[t])
        assert bool(d[0]) == bool(done[t]), t
        assert info["cost"][0] == cost[t], t
    env.close()


def ge_keys():
    g = load("golden_ground_effect.npz")
    return sorted({k.split("__")[0] + "__" + k.split("__")[1] for k in g.files})


def oracle_ge_from_golden(g, key, precision="f64", ground_effect=True):
    """Oracle env holding the reference drone's low-altitude start state, ground effect on."""
    c = build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", 1, observation_noise=0, domain_randomization=-1,
                     motor_thrust_noise=0, max_episode_steps=0, auto_reset=False)
    env = O.OracleEnv(c, precision)
    sf, si = env.get_state()
    sf[:] = 0
    sf[0:3, 0] = g[key + "__init_p"]; sf[3:7, 0] = g[key + "__init_q"]; sf[7:10, 0] = g[key + "__init_v"]
    sf[10:13, 0] = g[key + "__init_w"]; sf[16:20, 0] = g[key + "__init_x"]
    abuf = g[key + "__init_abuf"]
    for r in range(abuf.shape[0]):
        sf[24 + 4 * r:28 + 4 * r, 0] = abuf[r]
    sf[81, 0] = c.time_step; sf[82, 0] = c.mass; sf[83:86, 0] = (c.ixx, c.iyy, c.izz)
    sf[86, 0] = c.ft0; sf[87, 0] = c.ft1
    sf[88:92, 0] = c.A; sf[92:96, 0] = c.B; sf[96:100, 0] = c.K
    si[:] = 0
    env.set_state(sf, si)
    env.set_ground_effect(ground_effect)
    assert float(g[key + "__time_step"]) == c.time_step
    return env


@pytest.mark.parametrize("key", ge_keys())
def test_ground_effect_substeps_match_reference(key):
    """calculate_ground_effect + PyBulletPhysics.step_forward (physics.py:27-58, 91-124) with
    use_ground_effect=True, near the ground: every sub-step's p, q, v, w and motor state within
    1e-9 of the reference; ge__3 is flipped past |roll| = pi/2 (no ground effect, physics.py:55-58)."""
    g = load("golden_ground_effect.npz")
    acts, S = g[key + "__actions"], g[key + "__states"]
    env = oracle_ge_from_golden(g, key)
    off = oracle_ge_from_golden(g, key, ground_effect=False)
    for t in range(len(acts)):
        env.physics_step(acts[t:t + 1])
        off.physics_step(acts[t:t + 1])
        sf = env.get_state()[0][:, 0]
        got = np.concatenate([sf[0:13], sf[16:20] + sf[104:108]])
        err = np.abs(got - S[t]) / (1 + np.abs(S[t]))
        assert err.max() < 1e-9, (t, err.max(), np.argmax(err))
    dz = abs(env.get_state()[0][2, 0] - off.get_state()[0][2, 0])
    if key.endswith("3"):
        assert dz == 0.0                                  # flipped past pi/2: no ground effect
    else:
        assert dz > 1e-4                                  # the extra thrust near the ground shows
    env.close(); off.close()


HJ_ENV_IDS = {"DroneHoverBulletFreeEnvWithAdversary": "DroneHoverBulletFreeEnvWithAdversary-v0",
              "DroneHoverBulletEnvWithAdversary": "DroneHoverBulletEnvWithAdversary-v0",
              "DroneHoverBulletFreeEnvWithRandomHJAdversary": "DroneHoverBulletFreeEnvWithRandomHJAdversary-v0"}


def hj_golden_keys():
    g = load("golden_env_hj_trajectories.npz")
    return sorted({k.split("__")[0] + "__" + k.split("__")[1] for k in g.files})


def hj_oracle_from_golden(g, key, V, precision="f64"):
    name = key.split("__")[0]
    kw = {} if "Random" in name else dict(disturbance_level=float(g[key + "__level"]))
    return oracle_from_golden(g, key, HJ_ENV_IDS[name], precision, V=V, **kw)


@pytest.mark.parametrize("key", hj_golden_keys())
def test_hj_env_steps_match_reference(key, V):
    """The HJ-adversary env-step (hover_free.py:391-444, hover.py:649-702, the Boltzmann-level env
    hover_free.py:608-683): quat2euler + distur_gener on the state at the start of the step, only
    d[0], d[1] applied, then the env-step as in test_env_steps_match_reference."""
    g = load("golden_env_hj_trajectories.npz")
    env = hj_oracle_from_golden(g, key, V)
    acts, obs, rew, done, cost = (g[key + s] for s in ("__actions", "__obs", "__rew", "__done", "__cost"))
    assert len(acts) >= 10
    for t in range(len(acts)):
        o, r, d, info = env.step(acts[t:t + 1])
        err = np.abs(o[0] - obs[t]) / (1 + np.abs(obs[t]))
        assert err.max() < 1e-9, (t, err.max(), np.argmax(err))
        assert abs(r[0] - rew[t]) <= 1e-9 * (1 + abs(rew[t])), (t, r[0], rew[t])
        assert bool(d[0]) == bool(done[t]), t
        assert info["cost"][0] == cost[t], t
    env.close()


UNI_ENV_IDS = {"DroneHoverBulletFreeEnvWithRandomAdversary": "DroneHoverBulletFreeEnvWithRandomAdversary-v0",
               "DroneHoverBulletEnvWithRandomAdversary": "DroneHoverBulletEnvWithRandomAdversary-v0"}


def uniform_golden_keys():
    g = load("golden_env_uniform_trajectories.npz")
    return sorted({k.split("__")[0] + "__" + k.split("__")[1] for k in g.files})


@pytest.mark.parametrize("key", uniform_golden_keys())
def test_uniform_adversary_env_steps_match_reference(key):
    """The uniform-random-adversary env-step (hover_free.py:950-1007, hover.py:1208-1265) with
    each step's recorded dstb_space.sample() fed back as an external disturbance."""
    from cf2sim.config import DSTB_EXTERNAL
    g = load("golden_env_uniform_trajectories.npz")
    env = oracle_from_golden(g, key, UNI_ENV_IDS[key.split("__")[0]], disturbance=DSTB_EXTERNAL)
    acts, dstb, obs, rew, done, cost = (g[key + s] for s in ("__actions", "__dstb", "__obs", "__rew", "__done", "__cost"))
    assert len(acts) >= 10 and len(dstb) == len(acts)
    for t in range(len(acts)):
        o, r, d, info = env.step(acts[t:t + 1], dstb=dstb[t:t + 1])
        err = np.abs(o[0] - obs[t]) / (1 + np.abs(obs[t]))
        assert err.max() < 1e-9, (t, err.max(), np.argmax(err))
        assert abs(r[0] - rew[t]) <= 1e-9 * (1 + abs(rew[t])), (t, r[0], rew[t])
        assert bool(d[0]) == bool(done[t]), t
        assert info["cost"][0] == cost[t], t
    env.close()


RESET_FIELDS = (list(range(0, 13)) + list(range(16, 20)) + list(range(24, 32)) + [81, 82, 83, 84, 85, 86, 87]
                + list(range(92, 96)) + list(range(96, 100)))   # public snapshot rows of golden "names"


RESET_CASES = {"samples": "DroneHoverBulletFreeEnvWithoutAdversary-v0",
               "samples_hover": "DroneHoverBulletEnvWithoutAdversary-v0",
               "samples_initial": "DroneHoverBulletFreeEnvWithAdversaryInitial-v0",
               "samples_randomhj": "DroneHoverBulletFreeEnvWithRandomHJAdversary-v0"}


def reset_ks_pvalues(sf, key="samples"):
    """Two-sample Kolmogorov-Smirnov p-value per reset field: restated resets (sf [NF, N]) vs the
    reference's own reset() samples of one env class (golden_reset_samples.npz[key]); for the
    Boltzmann env also a chi-square test of the redrawn level's distribution."""
    from scipy.stats import chi2_contingency, ks_2samp
    g = load("golden_reset_samples.npz")
    ref, names = g[key].astype(np.float64), g["names"]
    assert ref.shape[1] == len(RESET_FIELDS)
    p = {str(names[k]): float(ks_2samp(sf[f], ref[:, k]).pvalue) for k, f in enumerate(RESET_FIELDS)}

    def rates(q, w):      # R(q) w: the sampled rpy_dot (hover_free.py:284-289 sets w = R^T rpy_dot)
        x, y, z, s_ = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - s_ * z), 2 * (x * z + s_ * y)],
                      [2 * (x * y + s_ * z), 1 - 2 * (x * x + z * z), 2 * (y * z - s_ * x)],
                      [2 * (x * z - s_ * y), 2 * (y * z + s_ * x), 1 - 2 * (x * x + y * y)]])
        return np.einsum("ijn,jn->in", R, w)
    mine, theirs = rates(sf[3:7], sf[10:13]), rates(ref[:, 3:7].T, ref[:, 10:13].T)
    for k in range(3):
        p[f"rate{k}"] = float(ks_2samp(mine[k], theirs[k]).pvalue)
    if key == "samples_randomhj":
        lv = np.round(np.asarray(g["levels_randomhj"]) * 10).astype(int)
        my = np.round(sf[103] * 10).astype(int)
        counts = np.stack([np.bincount(my, minlength=21)[:21], np.bincount(lv, minlength=21)[:21]])
        p["level"] = float(chi2_contingency(counts)[1])
    return p


@pytest.mark.parametrize("key", sorted(RESET_CASES))
def test_reset_distribution_matches_reference_samples(key):
    """DroneBaseEnv.reset + task_specific_reset + apply_domain_randomization (base.py:241-298,
    420-464; hover_free.py:237-289) is random in both implementations (numpy's MT19937 there,
    Philox here), so the pin is distributional: for each of the 41 pose / velocity / motor /
    action-ring / DR fields, 4000 restated resets and the reference's 3000 are one distribution
    (four env classes: free hover, hover, the pi/4 AdversaryInitial variant, the Boltzmann-level
    env with its redrawn level by a chi-square test)
    by a two-sample KS test (p > 1e-4), and so are the sampled body rates R(q) w (the R^T quirk of
    hover_free.py:284-289; the 0.028 kg K quirk shows up as p ~ 1e-220 if broken)."""
    c = build_config(RESET_CASES[key], 4000, seed=17)
    env = O.OracleEnv(c)
    env.reset()
    sf, _ = env.get_state()
    env.close()
    p = reset_ks_pvalues(sf, key)
    bad = {k: v for k, v in p.items() if v < 1e-4}
    assert not bad, bad
