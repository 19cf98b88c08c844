"""f3 batched rollout caller: GAE and the actor-critic against restatements of the reference's
own formulas (algs/core.py:105-110 discount_cumsum, :459-535 finish_path /
calculate_adv_and_value_targets, :228-291 MLPGaussianActor, algs/iwpg/iwpg.py:372-410 roll_out)."""
import math

import numpy as np
import pytest
import torch

from cf2sim.rollout import MLPActorCritic, collect, gae


def discount_cumsum(x, discount):
    """core.py:105-110 (scipy lfilter form), as an explicit backward loop."""
    out = np.zeros_like(x)
    acc = 0.0
    for t in range(len(x) - 1, -1, -1):
        acc = x[t] + discount * acc
        out[t] = acc
    return out


def reference_gae(rew, val, done, trunc, trunc_val, last_val, gamma, lam, rew_den=None):
    """roll_out + finish_path on one env's stream: an episode slice ends at done (bootstrap
    V(final obs) on a time-out, 0 on a terminal state) or at the end of the epoch (V(s_T)).
    rew_den: reward scaling, rewards clip(r / rew_den, -10, 10) (core.py:522-529)."""
    if rew_den is not None:
        rew = np.clip(np.asarray(rew, np.float64) / rew_den, -10.0, 10.0)
    T = len(rew)
    adv = np.zeros(T)
    start = 0
    for t in range(T):
        if done[t] or t == T - 1:
            last = (trunc_val[t] if trunc[t] else 0.0) if done[t] else last_val
            rews = np.append(rew[start:t + 1], last)
            vals = np.append(val[start:t + 1], last)
            deltas = rews[:-1] + gamma * vals[1:] - vals[:-1]
            adv[start:t + 1] = discount_cumsum(deltas, gamma * lam)
            start = t + 1
    return adv, adv + val


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_batched_gae_equals_per_episode_finish_path(seed):
    rng = np.random.default_rng(seed)
    T, N = 37, 23
    rew = rng.normal(size=(T, N))
    val = rng.normal(size=(T, N))
    done = rng.random((T, N)) < 0.1
    trunc = done & (rng.random((T, N)) < 0.4)
    trunc_val = rng.normal(size=(T, N))
    last_val = rng.normal(size=N)
    tt = lambda x: torch.as_tensor(x, dtype=torch.float64)
    adv, ret = gae(tt(rew), tt(val), torch.as_tensor(done), torch.as_tensor(trunc), tt(last_val), tt(trunc_val),
                   0.99, 0.95)
    for n in range(N):
        ra, rr = reference_gae(rew[:, n], val[:, n], done[:, n], trunc[:, n], trunc_val[:, n], last_val[n], 0.99, 0.95)
        np.testing.assert_allclose(adv[:, n].numpy(), ra, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(ret[:, n].numpy(), rr, rtol=1e-12, atol=1e-12)


def test_actor_critic_matches_reference_definitions():
    torch.manual_seed(0)
    ac = MLPActorCritic()
    assert [m.out_features for m in ac.pi_net if isinstance(m, torch.nn.Linear)] == [50, 50, 4]
    assert [m.out_features for m in ac.v_net if isinstance(m, torch.nn.Linear)] == [64, 64, 1]
    assert isinstance(ac.pi_net[1], torch.nn.ReLU) and isinstance(ac.v_net[1], torch.nn.Tanh)
    obs = torch.randn(128, 34)
    g = torch.Generator().manual_seed(1)
    a, v, logp = ac.step(obs, generator=g)
    mu = ac.pi_net(ac.normalize(obs)).detach()
    ref = torch.distributions.Normal(mu, torch.exp(ac.log_std)).log_prob(a).sum(-1)
    torch.testing.assert_close(logp, ref, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(v, ac.v_net(ac.normalize(obs)).squeeze(-1).detach())
    assert math.isclose(float(ac.log_std.exp()[0]), 0.5, rel_tol=1e-6)        # core.py:238
    ac.set_log_std(0.0)
    assert math.isclose(float(ac.log_std.exp()[0]), 0.01, rel_tol=1e-5)        # core.py:278
    a_det, _, _ = ac.step(obs, deterministic=True)
    torch.testing.assert_close(a_det, mu)


@pytest.mark.gpu
def test_collect_on_gpu_matches_reference_gae(gpu):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    torch.manual_seed(0)
    n, T = 512, 64
    envs = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithoutAdversary-v0", n, seed=5, want_final_obs=True,
                               max_episode_steps=20)                   # short limit: exercise time-outs
    ac = MLPActorCritic().to(gpu)
    g = torch.Generator(device=gpu).manual_seed(3)
    ro = collect(envs, ac, T, generator=g)
    assert ro.obs.shape == (T, n, 34) and ro.act.shape == (T, n, 4) and ro.adv.shape == (T, n)
    assert torch.isfinite(ro.adv).all() and torch.isfinite(ro.ret).all()
    d, tr = ro.done.cpu().numpy(), ro.trunc.cpu().numpy()
    assert tr.any() and (d & ~tr).any()                                  # both boundary kinds occur
    rew, val = ro.rew.double().cpu().numpy(), ro.val.double().cpu().numpy()
    adv = ro.adv.double().cpu().numpy()
    last_val, trunc_val = ro.last_val.double().cpu().numpy(), ro.trunc_val.double().cpu().numpy()
    torch.testing.assert_close(ro.last_val, ac.value(ro.last_obs))
    den = float(ac.ret_oms.std.item()) + 1e-5                         # reward scaling (IWPG default)
    for k in range(0, n, 7):
        ra, rr = reference_gae(rew[:, k], val[:, k], d[:, k], tr[:, k], trunc_val[:, k], last_val[k], 0.99, 0.95, den)
        np.testing.assert_allclose(adv[:, k], ra, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(ro.ret[:, k].double().cpu().numpy(), rr, rtol=1e-4, atol=1e-4)
    envs.close()


# mu / V tolerance vs the torch fp32 networks (mixed abs/rel |g - r| / (1 + |r|)) per product
# precision: fp32 MFMA differs from torch only in summation order and the v_exp/v_rcp tanh;
# bf16x3 adds <= ~1.1e-5 relative error per product (measured max over 3000 rows: see DESIGN.md 9)
POLICY_TOL = {"fp32": 2e-5, "bf16x3": 1.5e-4}


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
@pytest.mark.parametrize("obs_dim", [34, 42])
def test_fused_policy_matches_torch_networks(gpu, obs_dim, precision):
    """cf2_policy_forward vs the torch networks (fp32): mu and V within POLICY_TOL (mixed abs/rel),
    logp = Normal(mu, std).log_prob(act).sum(-1) exactly as the reference defines it, eps ~
    Philox normals keyed (seed, counter, row)."""
    import oracle as O
    from cf2sim.rollout import FusedActorCritic
    torch.manual_seed(obs_dim)
    ac = MLPActorCritic(obs_dim=obs_dim).to(gpu)
    for m in ac.modules():                       # non-trivial biases
        if isinstance(m, torch.nn.Linear):
            torch.nn.init.uniform_(m.bias, -0.3, 0.3)
    ac.obs_oms.update(torch.randn(5000, obs_dim, device=gpu) * torch.rand(obs_dim, device=gpu) * 4 + 1.0)
    fused = FusedActorCritic(ac, seed=1234, precision=precision)   # standardisation in the weight block
    n = 3000                                      # ragged last block
    obs = torch.randn(n, obs_dim, device=gpu) * 3
    with torch.no_grad():
        mu_ref = ac.pi_net(ac.normalize(obs))
        v_ref = ac.v_net(ac.normalize(obs)).squeeze(-1)
    a_det, v, _ = fused.step(obs, deterministic=True)
    err = lambda g, r: float(((g - r).abs() / (1 + r.abs())).max())
    print(f"{precision} D={obs_dim}: mu err {err(a_det, mu_ref):.2e}, v err {err(v, v_ref):.2e}")
    assert err(a_det, mu_ref) < POLICY_TOL[precision] and err(v, v_ref) < POLICY_TOL[precision]
    a, v2, logp = fused.step(obs)
    torch.testing.assert_close(v2, v)
    std = ac.log_std.exp()
    logp_ref = torch.distributions.Normal(mu_ref, std).log_prob(a).sum(-1)
    assert err(logp, logp_ref) < 1e-4
    eps = ((a - mu_ref) / std).cpu().numpy()
    for r in (0, 1, 255, 256, n - 1):            # eps = Box-Muller of Philox(seed, counter 1, row)
        u = O.philox([0, 1, r, 3], [1234, 0])
        u1 = ((u[0] >> 8) + 1.0) * 2.0 ** -24
        u2 = (u[1] >> 8) * 2.0 ** -24
        rad = math.sqrt(-2 * math.log(u1))
        np.testing.assert_allclose(eps[r, :2], [rad * math.cos(2 * math.pi * u2), rad * math.sin(2 * math.pi * u2)],
                                   atol=2e-4)


@pytest.mark.gpu
def test_fused_value_masked_and_collect(gpu):
    from cf2sim.rollout import FusedActorCritic
    from cf2sim.vec_env import BatchedCrazyflieEnv
    torch.manual_seed(0)
    ac = MLPActorCritic().to(gpu)
    fused = FusedActorCritic(ac, seed=9)
    obs = torch.randn(700, 34, device=gpu)
    mask = torch.rand(700, device=gpu) < 0.1
    out = torch.full((700,), -7.0, device=gpu)
    fused.value_masked(obs, mask, out)
    with torch.no_grad():
        v_ref = ac.value(obs)
    assert torch.all(out[~mask] == -7.0)
    assert float(((out[mask] - v_ref[mask]).abs() / (1 + v_ref[mask].abs())).max()) < 2e-5
    # sparse marks over many chunks (the collect-wide time-out pass), ragged row count, mask and
    # obs taken at an odd row offset
    rows = 300_007
    big = torch.randn(rows + 3, 34, device=gpu)[3:]
    mflag = torch.zeros(rows + 5, dtype=torch.uint8, device=gpu)[5:]
    idx = torch.cat([torch.tensor([0, 15, 16, rows - 1], device=gpu), torch.randint(0, rows, (60,), device=gpu)])
    mflag[idx] = 1
    out = torch.full((rows,), -7.0, device=gpu)
    fused.value_masked(big, mflag, out)
    sel = mflag.bool()
    with torch.no_grad():
        v_ref = ac.value(big[sel])
    assert torch.all(out[~sel] == -7.0)
    assert float(((out[sel] - v_ref).abs() / (1 + v_ref.abs())).max()) < 2e-5
    n, T = 512, 48
    envs = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithoutAdversary-v0", n, seed=5, want_final_obs=True,
                               max_episode_steps=20)
    ro = collect(envs, fused, T)
    d, tr = ro.done.cpu().numpy(), ro.trunc.cpu().numpy()
    assert tr.any() and torch.isfinite(ro.adv).all()
    rew, val = ro.rew.double().cpu().numpy(), ro.val.double().cpu().numpy()
    last_val, trunc_val = ro.last_val.double().cpu().numpy(), ro.trunc_val.double().cpu().numpy()
    # the time-out bootstraps equal the torch value of the pre-reset observation
    den = float(ac.ret_oms.std.item()) + 1e-5
    for k in range(0, n, 11):
        ra, _ = reference_gae(rew[:, k], val[:, k], d[:, k], tr[:, k], trunc_val[:, k], last_val[k], 0.99, 0.95, den)
        np.testing.assert_allclose(ro.adv[:, k].double().cpu().numpy(), ra, rtol=1e-4, atol=1e-4)
    envs.close()


@pytest.mark.gpu
def test_gae_kernel_matches_reference(gpu):
    from cf2sim.rollout import gae_device
    rng = np.random.default_rng(7)
    T, N = 29, 1000
    rew = rng.normal(size=(T, N)).astype(np.float32)
    val = rng.normal(size=(T, N)).astype(np.float32)
    done = rng.random((T, N)) < 0.1
    trunc = done & (rng.random((T, N)) < 0.4)
    trunc_val = rng.normal(size=(T, N)).astype(np.float32)
    last_val = rng.normal(size=N).astype(np.float32)
    g = lambda x: torch.as_tensor(x, device=gpu)
    adv, ret = gae_device(g(rew), g(val), g(done.astype(np.uint8)), g(trunc.astype(np.uint8)), g(last_val),
                          g(trunc_val), 0.99, 0.95)
    adv, ret = adv.cpu().numpy(), ret.cpu().numpy()
    for k in range(0, N, 13):
        ra, rr = reference_gae(rew[:, k].astype(np.float64), val[:, k].astype(np.float64), done[:, k], trunc[:, k],
                               trunc_val[:, k].astype(np.float64), float(last_val[k]), 0.99, 0.95)
        np.testing.assert_allclose(adv[:, k], ra, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(ret[:, k], rr, rtol=1e-4, atol=1e-4)


def test_return_std_host_mirror_follows_every_change():
    """collect() reads the return std on the host without a device sync per epoch (OnlineMeanStd.
    std_host caches it); the mirror must follow update(), in-place edits and a replaced buffer."""
    from cf2sim.rollout import OnlineMeanStd
    oms = OnlineMeanStd(shape=(1,))
    assert oms.std_host() == 1.0
    oms.update(torch.tensor([1.0, 3.0, 5.0]))
    assert oms.std_host() == pytest.approx(float(oms.std.item()))
    oms.std.fill_(2.5)
    assert oms.std_host() == 2.5
    oms.std = torch.full((1,), 4.0)
    assert oms.std_host() == 4.0
