"""The gym-style boundary: ids, spaces, the 4-tuple step API, TimeLimit semantics and the
physics-by-name plugin selection (phoenix_drone_simulation/__init__.py:8-109, envs/base.py:24,
139-148, 223-231, 466-507; tests/test_envs.py:96-123 is the reference's own check of this API)."""
import numpy as np
import pytest

import oracle as O
from cf2sim import registration as R
from cf2sim.config import OUT_OF_SCOPE_IDS, PHYS_BULLET, PHYS_SIMPLE, REFERENCE_IDS, build_config


def test_registry_holds_every_reference_hover_id():
    assert len(REFERENCE_IDS) == 11
    for env_id in REFERENCE_IDS:
        assert env_id in R.registry
    assert "DroneHoverBulletFreeEnvWithGust-v0" in R.registry       # BASELINE config C4 extension
    assert "DroneHoverBulletFreeEnvWithConstWind-v0" in R.registry  # BASELINE config C2 extension


@pytest.mark.parametrize("env_id", OUT_OF_SCOPE_IDS)
def test_out_of_scope_ids_fail_loudly(env_id):
    with pytest.raises(NotImplementedError):
        R.make(env_id)


def test_unknown_id_raises():
    with pytest.raises(KeyError):
        R.make("DroneHoverNoSuchEnv-v0")


def test_physics_plugin_names():
    assert R.resolve_physics(None, PHYS_BULLET) == PHYS_BULLET
    assert R.resolve_physics("HipBatchedPhysics", PHYS_SIMPLE) == PHYS_SIMPLE
    assert R.resolve_physics("SimplePhysics", PHYS_BULLET) == PHYS_SIMPLE
    assert R.resolve_physics("PybulletPhysicsWithAdversary", PHYS_SIMPLE) == PHYS_BULLET
    with pytest.raises(AssertionError):                 # envs/base.py:224-225
        R.resolve_physics("MuJoCoPhysics", PHYS_BULLET)


def test_make_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from cf2sim._native import CF2Error
    with pytest.raises(CF2Error):
        R.make("DroneHoverBulletEnv-v0")


@pytest.mark.gpu
@pytest.mark.parametrize("env_id", REFERENCE_IDS)
def test_make_step_api(gpu, env_id):
    """tests/test_envs.py:96-123 of the reference, through make(): obs in the observation space,
    4-tuple step with float reward, bool done and a dict info carrying the cost signal."""
    env = R.make(env_id, seed=1)
    if env._env.cfg.disturbance == 5:                  # HJ adversary: bind a (synthetic) value table
        import torch
        V = torch.zeros(1, 15 ** 6, device=gpu)
        env._env.bind_hj_tables(V, [0] * int(env._env.cfg.num_levels))
    if env._env.cfg.disturbance == 1:                  # external dstb: not a single-env gym API
        env.close()
        pytest.skip("external-disturbance envs take dstb via BatchedCrazyflieEnv.step")
    obs = env.reset()
    assert obs.dtype == np.float64 and obs.shape == env.observation_space.shape
    assert env.observation_space.contains(obs.astype(np.float32))
    for _ in range(5):
        a = env.action_space.sample()
        obs, r, done, info = env.step(a)
        assert isinstance(r, float) and isinstance(done, bool) and isinstance(info, dict)
        assert "cost" in info and "disturbance_level" in info
        assert obs.shape == env.observation_space.shape
        if done:
            obs = env.reset()
    env.close()


@pytest.mark.gpu
def test_make_matches_restatement_and_time_limit(gpu):
    """One env through make() == the fp32 restatement with the same seed (env id 0 of the Philox
    stream), and gym's TimeLimit(max_episode_steps) ends the episode with TimeLimit.truncated."""
    env_id = "DroneHoverBulletFreeEnvWithoutAdversary-v0"
    env = R.make(env_id, seed=7, max_episode_steps=40)
    ref = O.OracleEnv(build_config(env_id, 1, seed=7, auto_reset=False, max_episode_steps=0), precision="f32")
    o_g, o_r = env.reset(), ref.reset()[0]
    assert np.max(np.abs(o_g - o_r) / (1 + np.abs(o_r))) < 2e-5
    a = np.full(4, 0.1111, dtype=np.float32)          # near hover: the episode survives 40 steps
    for t in range(40):
        o_g, r_g, d_g, info = env.step(a)
        o_r, r_r, d_r, _ = ref.step(a[None])
        assert np.max(np.abs(o_g - o_r[0]) / (1 + np.abs(o_r[0]))) < 5e-4, t
        assert abs(r_g - float(r_r[0])) < 1e-3
        # the penalty terms the reference logs (hover_free.py:227-232) add up to the reward
        assert abs(r_g + env.penalty_log + env.penalty_z_log) < 1e-4 * (1 + abs(r_g))
        assert env.penalty_rpy_log >= 0 and env.penalty_rpy_dot_log >= 0 and env.penalty_velocity_log >= 0
        assert not bool(d_r[0])
        assert d_g == (t == 39)
    assert info.get("TimeLimit.truncated") is True
    with pytest.raises(RuntimeError):
        env.step(a)
    env.close()
    ref.close()


@pytest.mark.gpu
def test_make_step_cost_is_recorded(gpu):
    """The single-env adapter's per-step cost (the reference's batch-1 callers, algs/iwpg/iwpg.py:380,
    go through it): one kernel, one state snapshot and ONE device->host transfer per step.  The
    figure is written to gpurun_out/make_step_us.json (DESIGN.md quotes it)."""
    import json
    import os
    import time
    env = R.make("DroneHoverBulletFreeEnvWithoutAdversary-v0", seed=3)
    env.reset()
    a = np.full(4, 0.1111, dtype=np.float32)
    for _ in range(20):
        _, _, d, _ = env.step(a)
        if d:
            env.reset()
    n, t0 = 300, time.perf_counter()
    for _ in range(n):
        _, _, d, _ = env.step(a)
        if d:
            env.reset()
    us = (time.perf_counter() - t0) / n * 1e6
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "make_step_us.json"), "w") as f:
        json.dump({"us_per_make_step": us, "steps": n}, f)
    env.close()
    assert us < 2000.0, f"{us:.0f} us per make().step()"
