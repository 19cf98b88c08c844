"""cf2_rollout: K env-steps fused in one launch (state in registers) must equal K cf2_step calls
with the same actions -- observations, rewards, dones, truncations, costs, levels, final
observations and the state afterwards -- across auto-resets, TimeLimit truncations, the noise /
DR / gust / HJ / formation paths and launches that the host splits into residency slices."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [
    ("DroneHoverBulletFreeEnvWithGust-v0", 3000, {}),
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", 1024, dict(max_episode_steps=7)),
    ("DroneHoverSimpleEnv-v0", 777, {}),
    ("DroneHoverBulletFreeEnvWithConstWind-v0", 512, dict(observation_noise=0)),
    ("DroneHoverBulletFreeEnvWithDownwash-v0", 1024, {}),
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", 512, dict(aggregate_phy_steps=1, latency=0.02, max_episode_steps=9)),
    ("DroneHoverBulletFreeEnvWithGust-v0", 150000, {}),       # > one residency round: sliced
]


@pytest.mark.parametrize("env_id,n,kw", CASES)
def test_fused_rollout_equals_step_loop(gpu, env_id, n, kw):
    _compare(gpu, env_id, n, kw)


@pytest.mark.parametrize("n", [2000, 40000])
def test_fused_rollout_boltzmann_hj_levels(gpu, n):
    """The Boltzmann-level HJ env: a reset redraws the episode's level, which the small-N
    rollout's helper waves track from step to step for their speculative resets."""
    from test_gpu_parity import _synthetic_tables
    V = torch.from_numpy(_synthetic_tables(tuple(range(3)), seed=1)).cuda()
    tol = [lv % 3 for lv in range(21)]
    _compare(gpu, "DroneHoverBulletFreeEnvWithRandomHJAdversary-v0", n, dict(max_episode_steps=6),
             setup=lambda e: e.bind_hj_tables(V, tol))


def _compare(gpu, env_id, n, kw, setup=None):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    K = 24
    a = (torch.rand(K, n, 4, device=gpu, generator=torch.Generator(device=gpu).manual_seed(3)) * 2 - 1).contiguous()
    ref = BatchedCrazyflieEnv(env_id, n, seed=9, want_final_obs=True, **kw)
    fus = BatchedCrazyflieEnv(env_id, n, seed=9, want_final_obs=True, **kw)
    if setup is not None:
        setup(ref)
        setup(fus)
    ref.reset()
    fus.reset()
    outs = {k: [] for k in ("obs", "rew", "done", "trunc", "cost", "level", "fin")}
    for k in range(K):
        o, r, d, info = ref.step(a[k])
        for key, t in (("obs", o), ("rew", r), ("done", d), ("trunc", info["truncated"]), ("cost", info["cost"]),
                       ("level", info["disturbance_level"]), ("fin", info["final_obs"])):
            outs[key].append(t.clone())
    o, r, d, info = fus.rollout(a)
    done = torch.stack(outs["done"]).bool()
    assert done.any(), "no auto-reset inside the window"
    torch.testing.assert_close(d, torch.stack(outs["done"]), rtol=0, atol=0)
    torch.testing.assert_close(info["truncated"], torch.stack(outs["trunc"]), rtol=0, atol=0)
    for key, got in (("obs", o), ("rew", r), ("cost", info["cost"]), ("level", info["disturbance_level"])):
        torch.testing.assert_close(got, torch.stack(outs[key]), rtol=1e-6, atol=1e-6, msg=key)
    fin = info["final_obs"][done]
    torch.testing.assert_close(fin, torch.stack(outs["fin"])[done], rtol=1e-6, atol=1e-6)
    gs, gi = fus.get_state()
    rs, ri = ref.get_state()
    torch.testing.assert_close(gi, ri, rtol=0, atol=0)
    torch.testing.assert_close(gs, rs, rtol=1e-6, atol=1e-6)
    # continuing with single steps from the rollout's final state stays identical
    b = torch.rand(n, 4, device=gpu) * 2 - 1
    o1 = ref.step(b)[0].clone()
    o2 = fus.step(b)[0]
    torch.testing.assert_close(o2, o1, rtol=1e-6, atol=1e-6)
    ref.close()
    fus.close()


def test_rollout_rejects_bad_buffers(gpu):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithoutAdversary-v0", 64)
    env.reset()
    with pytest.raises(ValueError):
        env.rollout(torch.zeros(4, 63, 4, device=gpu))
    with pytest.raises(ValueError):
        env.rollout(torch.zeros(4, 64, 4, device=gpu, dtype=torch.float64))
    env.close()
