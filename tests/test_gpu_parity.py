"""Parity of the HIP kernels (through the C ABI) against the CPU restatement (oracle/).

Errors are mixed abs/rel: |gpu - ref| / (1 + |ref|).  Tolerances (stated per test):
* vs the fp32 restatement (same formulas in fp32; the kernel additionally contracts FMAs and
  uses the hardware sin/cos/log/sqrt/rcp, ~1-2 ulp): 5e-4 on observations and on the stored
  state over 120 env-steps with sensor noise, DR and auto-resets (the largest differences are
  angular rates of tumbling envs, where ulp-level differences grow chaotically);
* vs the fp64 restatement: fp32 rounding of the whole trajectory -> 5e-3 on observations
  over 120 env-steps (BASELINE.json's "1e-4 rel" is checked closed-loop, test below);
* integer/boolean outputs (done, truncation, episode counters, RNG counters): exact, except
  envs whose trajectory crosses a termination threshold within fp32 rounding;
* re-synchronised (the restatement loaded with the kernel's state before every env-step, so one
  step's rounding is all that can separate them): 2e-5 on observations, 1e-5 on rewards, done and
  truncation exact, no exemption.
"""
import numpy as np
import pytest
import torch

import oracle as O
from cf2sim.config import build_config
from parity_util import CLEAN, STATE_BLOCKS, pd_actions, state_rel_err  # noqa: F401

pytestmark = pytest.mark.gpu

CASES = [
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", {}),
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(observation_noise=0, domain_randomization=-1,
                                                         motor_thrust_noise=0)),
    ("DroneHoverSimpleEnv-v0", {}),
    ("DroneHoverBulletEnvWithRandomAdversary-v0", {}),
    ("DroneHoverBulletFreeEnvWithGust-v0", {}),
    ("DroneHoverBulletFreeEnvWithConstWind-v0", {}),
    ("DroneHoverBulletEnv-v0", dict(observation_noise=0)),
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(aggregate_phy_steps=1)),   # held obs persists
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(latency=0.02)),           # ring of 4
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(latency=0.0)),            # no latency
]


def _actions(rng, n):
    return (rng.uniform(-1, 1, size=(n, 4)) * 0.25 + 0.1111).astype(np.float32)


def _run_pair(env_id, kw, n, T, prec, seed=3, stop_at_done=False):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env = BatchedCrazyflieEnv(env_id, n, seed=seed, want_final_obs=True, **kw)
    ref = O.OracleEnv(build_config(env_id, n, seed=seed, **kw), precision=prec)
    go = env.reset().cpu().numpy()
    ro = ref.reset()
    def nerr(g, r):   # mixed abs/rel error: |g - r| / (1 + |r|)
        return float((np.abs(g - r) / (1.0 + np.abs(r))).max()) if g.size else 0.0
    errs = [nerr(go, ro)]
    rng = np.random.default_rng(seed + 1)
    done_mismatch = 0
    rew_err = 0.0
    for t in range(T):
        a = _actions(rng, n)
        g_o, g_r, g_d, g_i = env.step(torch.from_numpy(a).cuda())
        r_o, r_r, r_d, r_i = ref.step(a, want_final=True)
        g_o, g_d = g_o.cpu().numpy(), g_d.cpu().numpy().astype(bool)
        done_mismatch += int((g_d != r_d).sum())
        errs.append(nerr(g_o, r_o))
        rew_err = max(rew_err, float(np.abs(g_r.cpu().numpy() - r_r).max()))
        fin = g_i["final_obs"].cpu().numpy()
        m = r_d & g_d
        if m.any():
            errs[-1] = max(errs[-1], nerr(fin[m], r_i["final_obs"][m]))
        np.testing.assert_array_equal(g_i["truncated"].cpu().numpy().astype(bool) & ~(g_d != r_d), r_i["truncated"] & ~(g_d != r_d))
    gsf, gsi = env.get_state()
    rsf, rsi = ref.get_state()
    env.check_device_errors()          # no helper wave gave up on an LDS hand-over
    env.close()
    ref.close()
    return np.array(errs), done_mismatch, rew_err, (gsf.cpu().numpy(), gsi.cpu().numpy()), (rsf, rsi)


@pytest.mark.parametrize("env_id,kw", CASES)
def test_kernel_matches_fp32_restatement(gpu, env_id, kw):
    n, T = 512, 120
    errs, dmis, rew_err, (gsf, gsi), (rsf, rsi) = _run_pair(env_id, kw, n, T, "f32")
    assert errs[0] < 2e-5, f"reset observation {errs[0]}"
    assert errs.max() < 5e-4, f"obs max err {errs.max()}"
    assert dmis == 0
    assert rew_err < 2e-3 * 1000 / 1000 + 1e-3
    np.testing.assert_array_equal(gsi[0], rsi[0])   # episode steps
    np.testing.assert_array_equal(gsi[1], rsi[1])   # RNG counters
    ol = 13 if kw.get("observation_noise", 1) > 0 else 17
    fields = list(range(0, 13)) + list(range(16, 24)) + list(range(56, 56 + ol)) + list(range(73, 81))
    fe = (np.abs(gsf[fields] - rsf[fields]) / (1 + np.abs(rsf[fields]))).max(1)
    top = sorted(zip(fe.tolist(), fields), reverse=True)[:4]
    assert fe.max() < 5e-4, "state field errors (err, field): " + repr(top)


@pytest.mark.parametrize("env_id,kw", CASES)
def test_kernel_matches_fp32_restatement_resynchronised(gpu, env_id, kw):
    """The strict form of the test above: before every env-step the restatement is loaded with the
    kernel's own state (cf2_get_state -> OracleEnv.set_state), so each of the 120 env-steps is
    compared from identical bits and no chaotic growth can hide behind the 5e-4 band: every
    observation within 2e-5 mixed abs/rel, rewards within 1e-5 (relative to 1 + |r|), done and
    truncation exact, across auto-resets."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n, T, seed = 512, 120, 3
    env = BatchedCrazyflieEnv(env_id, n, seed=seed, want_final_obs=True, **kw)
    ref = O.OracleEnv(build_config(env_id, n, seed=seed, **kw), precision="f32")
    env.reset()
    ref.reset()
    rng = np.random.default_rng(seed + 1)
    worst_o = worst_r = 0.0
    dones = 0
    for t in range(T):
        gsf, gsi = env.get_state()
        ref.set_state(gsf.cpu().numpy(), gsi.cpu().numpy())
        a = _actions(rng, n)
        g_o, g_r, g_d, g_i = env.step(torch.from_numpy(a).cuda())
        r_o, r_r, r_d, r_i = ref.step(a, want_final=True)
        g_o, g_r = g_o.cpu().numpy(), g_r.cpu().numpy()
        worst_o = max(worst_o, float((np.abs(g_o - r_o) / (1.0 + np.abs(r_o))).max()))
        worst_r = max(worst_r, float((np.abs(g_r - r_r) / (1.0 + np.abs(r_r))).max()))
        np.testing.assert_array_equal(g_d.cpu().numpy().astype(bool), r_d)
        np.testing.assert_array_equal(g_i["truncated"].cpu().numpy().astype(bool), r_i["truncated"])
        dones += int(r_d.sum())
    env.check_device_errors()
    env.close()
    ref.close()
    assert worst_o < 2e-5, worst_o
    assert worst_r < 1e-5, worst_r
    assert dones > 0


@pytest.mark.parametrize("env_id,kw", CASES[:3])
def test_kernel_tracks_fp64_restatement(gpu, env_id, kw):
    errs, dmis, rew_err, (gsf, gsi), (rsf, rsi) = _run_pair(env_id, kw, 512, 120, "f64")
    assert errs.max() < 5e-3
    assert dmis <= 2


def _closed_loop(kw, n=256, T=240, seed=11):
    env_id = "DroneHoverBulletFreeEnvWithoutAdversary-v0"
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env = BatchedCrazyflieEnv(env_id, n, seed=seed, **kw)
    cfg = build_config(env_id, n, seed=seed, **kw)
    ref = O.OracleEnv(cfg, "f64")
    sl = slice(21, 34) if kw.get("observation_noise", 1) <= 0 else slice(17, 30)   # o_k: p, q, v, w
    go = env.reset().cpu().numpy()
    ro = ref.reset()
    alive = np.ones(n, bool)
    for _ in range(T):
        go, _, _, _ = env.step(torch.from_numpy(pd_actions(go[:, sl], cfg.hover_action)).cuda())
        go = go.cpu().numpy()
        ro, _, rd, _ = ref.step(pd_actions(ro[:, sl], cfg.hover_action))
        alive &= ~rd
    g = env.get_state()[0].cpu().numpy()[:13].astype(np.float64)
    r = ref.get_state()[0][:13]
    env.close()
    ref.close()
    return g, r, alive


def test_closed_loop_state_within_1e4_rel_over_240_steps(gpu):
    """BASELINE.json: "state within 1e-4 rel of PyBullet over 240 steps", against the fp64
    restatement (the Bullet step itself is restated, PyBullet is absent: parity vs PyBullet
    unpinned).  A PD controller closes the loop on each env's own
    observation, as a policy does.  Noise-free config: every state vector < 1e-4 (state_rel_err)
    and also every one of the 13 components < 1e-4 relative to max(|x|, 1).  Measured on the fp32
    restatement with the compensated motor state: 4.3e-5 norm-wise, 5.1e-5 per component
    (1.4e-4 per component before the motor-state compensation)."""
    g, r, alive = _closed_loop(CLEAN)
    assert alive.all()
    errs = state_rel_err(g, r)
    worst = {k: float(v.max()) for k, v in errs.items()}
    assert max(worst.values()) < 1e-4, worst
    comp = np.abs(g - r) / np.maximum(np.abs(r), 1.0)
    assert comp.max() < 1e-4, comp.max(1)


def test_kernel_no_further_from_fp64_than_the_reference_algebra_in_fp32(gpu):
    """The fp32 suite above compares the kernel with an fp32 restatement that carries the kernel's
    own compensated motor recurrence; here the comparison is also made with the reference's own
    algebra in fp32 (oracle f32ref: x = A x + B u, envs/agents.py:287-288, rounded every sub-step).
    Closed loop over 240 env-steps (a PD controller on each side's own observation), the
    reference-default config: the kernel's state is at least as close to the fp64 restatement as
    the literal fp32 transcription of the reference is, and within 1e-3 of that transcription."""
    env_id = "DroneHoverBulletFreeEnvWithoutAdversary-v0"
    kw = dict(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0)
    n, T, seed = 256, 240, 11
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env = BatchedCrazyflieEnv(env_id, n, seed=seed, **kw)
    cfg = build_config(env_id, n, seed=seed, **kw)
    ref64, ref32 = O.OracleEnv(cfg, "f64"), O.OracleEnv(cfg, "f32ref")
    sl = slice(21, 34)
    go, r64, r32 = env.reset().cpu().numpy(), ref64.reset(), ref32.reset()
    alive = np.ones(n, bool)
    for _ in range(T):
        go = env.step(torch.from_numpy(pd_actions(go[:, sl], cfg.hover_action)).cuda())[0].cpu().numpy()
        r64, _, d64, _ = ref64.step(pd_actions(r64[:, sl], cfg.hover_action))
        r32, _, d32, _ = ref32.step(pd_actions(r32[:, sl], cfg.hover_action))
        alive &= ~d64 & ~d32
    g = env.get_state()[0].cpu().numpy()[:13].astype(np.float64)
    s64, s32 = ref64.get_state()[0][:13], ref32.get_state()[0][:13]
    env.close()
    ref64.close()
    ref32.close()
    assert alive.sum() >= n // 2
    def worst(a, b):
        return max(float(v.max()) for v in state_rel_err(a[:, alive], b[:, alive]).values())
    e_kernel, e_ref32, e_pair = worst(g, s64), worst(s32, s64), worst(g, s32)
    assert e_kernel <= 1.2 * e_ref32 + 1e-7, (e_kernel, e_ref32)
    assert e_pair < 1e-3, e_pair


def test_closed_loop_noisy_dr_state_within_1e4_rel_over_240_steps(gpu):
    """The same target on the reference-default config (sensor noise, 10 % DR, motor-thrust OU
    noise, latency): the PD loop acts on the noisy observation; both sides draw the same Philox
    noise.  Every state vector < 1e-4 (state_rel_err).  Measured on the fp32 restatement: 3.5e-5."""
    g, r, alive = _closed_loop(dict(max_episode_steps=0))
    errs = state_rel_err(g, r)
    worst = {k: float(v.max()) for k, v in errs.items()}
    assert max(worst.values()) < 1e-4, worst


def test_open_loop_replay_state_within_1e4_rel_over_240_steps(gpu):
    """Open loop: one fixed sequence of near-hover actions (hover + 0.02 N(0, 1)) replayed on the
    kernel and on the fp64 restatement for 240 env-steps from the same random resets (noise-free
    config).  Every state vector < 1e-4 (state_rel_err); measured on the fp32 restatement 5.1e-5."""
    env_id = "DroneHoverBulletFreeEnvWithoutAdversary-v0"
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = 256
    env = BatchedCrazyflieEnv(env_id, n, seed=11, **CLEAN)
    cfg = build_config(env_id, n, seed=11, **CLEAN)
    ref = O.OracleEnv(cfg, "f64")
    env.reset()
    ref.reset()
    rng = np.random.default_rng(0)
    for _ in range(240):
        a = (cfg.hover_action + 0.02 * rng.standard_normal((n, 4))).astype(np.float32)
        env.step(torch.from_numpy(a).cuda())
        ref.step(a)
    g = env.get_state()[0].cpu().numpy()[:13].astype(np.float64)
    r = ref.get_state()[0][:13]
    env.close()
    ref.close()
    worst = {k: float(v.max()) for k, v in state_rel_err(g, r).items()}
    assert max(worst.values()) < 1e-4, worst


def test_reset_mask_and_state_round_trip(gpu):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env_id = "DroneHoverBulletFreeEnvWithoutAdversary-v0"
    n = 300
    env = BatchedCrazyflieEnv(env_id, n, seed=21)
    ref = O.OracleEnv(build_config(env_id, n, seed=21), "f32")
    env.reset(); ref.reset()
    rng = np.random.default_rng(0)
    for t in range(5):
        a = _actions(rng, n)
        env.step(torch.from_numpy(a).cuda()); ref.step(a)
    mask = (np.arange(n) % 3 == 0).astype(np.uint8)
    go = env.reset(torch.from_numpy(mask).cuda()).cpu().numpy()
    ro = ref.reset(mask)
    m = mask.astype(bool)
    assert np.abs(go[m] - ro[m]).max() < 1e-5
    sf, si = env.get_state()
    env2 = BatchedCrazyflieEnv(env_id, n, seed=21)
    env2.set_state(sf, si)
    a = torch.from_numpy(_actions(rng, n)).cuda()
    o1 = env.step(a)[0].clone()
    o2 = env2.step(a)[0].clone()
    assert torch.equal(o1, o2)


def test_time_limit_truncation_on_gpu(gpu):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    kw = dict(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0, enable_reset_distribution=False,
              max_episode_steps=7)
    env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithoutAdversary-v0", 64, seed=0, **kw)
    env.reset()
    a = torch.full((64, 4), 0.1111111, device="cuda")
    for k in range(7):
        o, r, d, info = env.step(a)
    assert bool(d.all()) and bool(info["truncated"].all())
    sf, si = env.get_state()
    assert int(si[0].max()) == 0


def _synthetic_tables(levels=(0.0, 1.5), seed=0):
    """Smooth random HJ-like value tables over the 15^6 grid (float32, C-order)."""
    rng = np.random.default_rng(seed)
    axes = [np.linspace(-1, 1, 15) for _ in range(6)]
    out = []
    for li, _ in enumerate(levels):
        c = rng.normal(size=6)
        g = [a.reshape([-1 if i == d else 1 for i in range(6)]) for d, a in enumerate(axes)]
        V = sum(c[d] * g[d] ** (1 + (d % 2)) for d in range(6)) + 0.1 * np.sin(3 * g[3] + 2 * g[4] - g[5])
        V = V + 0.01 * rng.normal(size=(15,) * 6)
        out.append(V.astype(np.float32))
    return np.stack(out)


def test_hj_disturbance_batched_matches_restatement(gpu):
    from cf2sim.vec_env import hj_disturbance
    c = build_config("DroneHoverBulletFreeEnvWithAdversary-v0", 1)
    V = _synthetic_tables((1.5,))[0]
    rng = np.random.default_rng(2)
    n = 20000
    s = np.concatenate([rng.uniform(-1.6, 1.6, (n, 3)), rng.uniform(-4, 4, (n, 3))], 1).astype(np.float32)
    # grid nodes and mid-points exercise the tie rule and the boundary rows
    from cf2sim.config import hj_grid
    _, _, pts = hj_grid()
    s[:200, 3] = pts[3][rng.integers(0, 15, 200)]
    s[200:400, 4] = 0.5 * (pts[4][:-1] + pts[4][1:])[rng.integers(0, 14, 200)]
    u, d = hj_disturbance(torch.from_numpy(V).cuda(), torch.from_numpy(s).cuda(), 1.5, c)
    rd, ru, _ = O.hj(c, V, s.astype(np.float64), 1.5)
    np.testing.assert_array_equal(d.cpu().numpy(), rd.astype(np.float32))
    np.testing.assert_array_equal(u.cpu().numpy(), ru.astype(np.float32))


@pytest.mark.parametrize("env_id", ["DroneHoverBulletFreeEnvWithAdversary-v0",
                                    "DroneHoverBulletFreeEnvWithRandomHJAdversary-v0"])
def test_hj_adversary_env_matches_restatement(gpu, env_id):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    c = build_config(env_id, 256, seed=4)
    levels = 21
    V = _synthetic_tables(tuple(range(3)), seed=1)
    table_of_level = [l % 3 for l in range(levels)]
    env = BatchedCrazyflieEnv(env_id, 256, seed=4)
    env.bind_hj_tables(torch.from_numpy(V).cuda(), table_of_level)
    ref = O.OracleEnv(c, "f32")
    ref.bind_tables(V, table_of_level)
    env.reset(); ref.reset()
    rng = np.random.default_rng(9)
    for t in range(60):
        a = _actions(rng, 256)
        go, gr, gd, gi = env.step(torch.from_numpy(a).cuda())
        ro, rr, rd, ri = ref.step(a)
        assert np.abs(go.cpu().numpy() - ro).max() < 5e-4
        np.testing.assert_allclose(gi["disturbance_level"].cpu().numpy(), ri["level"], atol=1e-6)


@pytest.mark.parametrize("kw", [{}, dict(latency=0.02)])      # SPEC 2 (default shape) and the generic path
def test_downwash_formations_match_restatement(gpu, kw):
    """4-drone formations with downwash (f4).  The downwash force is a Gaussian in the horizontal
    offset with a 5 cm width (beta = 0.16 dz - 0.11 at dz = 1 m), so ulp-level differences
    (FMA contraction, v_rcp / v_exp) are amplified chaotically: the horizon is 25 env-steps,
    within which the trajectories must agree to the same 5e-4 as the single-drone cases."""
    errs, dmis, rew_err, (gsf, gsi), (rsf, rsi) = _run_pair("DroneHoverBulletFreeEnvWithDownwash-v0", kw, 512, 25, "f32")
    assert errs[0] < 2e-5, f"reset observation {errs[0]}"
    assert errs.max() < 5e-4, f"obs max err {errs.max()} {errs}"
    assert dmis == 0


@pytest.mark.parametrize("n", [1, 63, 300, 1000])
def test_ragged_env_counts_match_restatement(gpu, n):
    """Env counts that fill no whole wave / block (the kernel's tail guards, the per-block reset
    lists and the coalesced obs copy of a partial block) vs the fp32 restatement: 150 env-steps of
    the noisy, domain-randomised gust env with wide actions, so auto-resets hit partial blocks."""
    env_id = "DroneHoverBulletFreeEnvWithGust-v0"
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env = BatchedCrazyflieEnv(env_id, n, seed=21, want_final_obs=True)
    ref = O.OracleEnv(build_config(env_id, n, seed=21), precision="f32")
    go, ro = env.reset().cpu().numpy(), ref.reset()
    assert float((np.abs(go - ro) / (1 + np.abs(ro))).max()) < 2e-5
    rng = np.random.default_rng(5)
    resets = 0
    for t in range(150):
        a = (rng.uniform(-1, 1, size=(n, 4)) * 0.6 + 0.1111).astype(np.float32)
        g_o, g_r, g_d, g_i = env.step(torch.from_numpy(a).cuda())
        r_o, r_r, r_d, r_i = ref.step(a, want_final=True)
        g_d = g_d.cpu().numpy().astype(bool)
        np.testing.assert_array_equal(g_d, r_d)
        resets += int(r_d.sum())
        err = float((np.abs(g_o.cpu().numpy() - r_o) / (1 + np.abs(r_o))).max())
        assert err < 5e-4, (t, err)
        assert float(np.abs(g_r.cpu().numpy() - r_r).max()) < 3e-3
        if r_d.any():
            fin = g_i["final_obs"].cpu().numpy()[r_d]
            assert float((np.abs(fin - r_i["final_obs"][r_d]) / (1 + np.abs(r_i["final_obs"][r_d]))).max()) < 5e-4
    gsi, rsi = env.get_state()[1].cpu().numpy(), ref.get_state()[1]
    np.testing.assert_array_equal(gsi[:2], rsi[:2])        # episode steps, RNG counters
    env.close(); ref.close()
    assert n < 63 or resets > 0


def test_zero_envs_is_rejected(gpu):
    """An empty batch is an invalid configuration (cf2_create returns CF2_ERR_INVALID_ARG)."""
    from cf2sim._native import CF2Error
    from cf2sim.vec_env import BatchedCrazyflieEnv
    with pytest.raises((CF2Error, ValueError)):
        BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithoutAdversary-v0", 0)


def test_downwash_formations_long_horizon_closed_loop(gpu):
    """f4 over 240 env-steps (round-2 review: the 25-step horizon above is short).  Closed loop:
    every drone's PD controller acts on its own observation, on the HIP kernel and on the fp32
    restatement, so the formations keep flying.  The 5 cm downwash Gaussian amplifies ulp-level
    differences chaotically in a few formations whose drones pass through each other's wake, so
    the bound is on the distribution over drones (still flying on both sides), not on its maximum:
    at every 20th env-step the median error stays < 2e-5 and >= 93 % of the drones within 5e-4
    (measured: median 8e-7 -> 9e-6, 96-100 % within 5e-4; tests/diag_downwash_horizon.py)."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env_id, n, T = "DroneHoverBulletFreeEnvWithDownwash-v0", 512, 240
    env = BatchedCrazyflieEnv(env_id, n, seed=3, want_final_obs=True)
    cfg = build_config(env_id, n, seed=3)
    ref = O.OracleEnv(cfg, precision="f32")
    go, ro = env.reset().cpu().numpy(), ref.reset()
    alive = np.ones(n, bool)
    for t in range(T):
        g_o, _, g_d, _ = env.step(torch.from_numpy(pd_actions(go[:, 17:30], cfg.hover_action)).cuda())
        r_o, _, r_d, _ = ref.step(pd_actions(ro[:, 17:30], cfg.hover_action))
        go, ro = g_o.cpu().numpy(), r_o
        alive &= ~g_d.cpu().numpy().astype(bool) & ~r_d
        if (t + 1) % 20 == 0:
            e = (np.abs(go - ro) / (1 + np.abs(ro))).max(1)[alive]
            assert alive.sum() >= 150, (t, int(alive.sum()))
            assert float(np.median(e)) < 2e-5, (t, float(np.median(e)))
            assert float((e < 5e-4).mean()) >= 0.93, (t, float((e < 5e-4).mean()))
    env.close()
    ref.close()


def test_downwash_formations_resynchronised_every_step(gpu):
    """The strict form of the long-horizon test above, with no drone exempt: the same 240
    closed-loop env-steps, but before every env-step the restatement is loaded with the kernel's
    own state (cf2_get_state -> OracleEnv.set_state), so the chaotic wake crossings cannot
    accumulate ulp differences and each step is compared from identical bits.  Every drone of every
    env-step: observation within 2e-5 mixed abs/rel, done exact."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env_id, n, T = "DroneHoverBulletFreeEnvWithDownwash-v0", 512, 240
    env = BatchedCrazyflieEnv(env_id, n, seed=3)
    cfg = build_config(env_id, n, seed=3)
    ref = O.OracleEnv(cfg, precision="f32")
    go = env.reset().cpu().numpy()
    ref.reset()
    worst, dones = 0.0, 0
    for t in range(T):
        gsf, gsi = env.get_state()
        ref.set_state(gsf.cpu().numpy(), gsi.cpu().numpy())
        a = pd_actions(go[:, 17:30], cfg.hover_action)
        g_o, _, g_d, _ = env.step(torch.from_numpy(a).cuda())
        r_o, _, r_d, _ = ref.step(a)
        go = g_o.cpu().numpy()
        worst = max(worst, float((np.abs(go - r_o) / (1 + np.abs(r_o))).max()))
        np.testing.assert_array_equal(g_d.cpu().numpy().astype(bool), r_d)
        dones += int(r_d.sum())
    assert worst < 2e-5, worst
    env.check_device_errors()
    env.close()
    ref.close()
