"""f3 pinned on the reference's own learner code: tests/golden/golden_f3.npz was produced by
tests/golden/make_golden_f3.py running phoenix_drone_simulation/algs/core.py (discount_cumsum,
ActorCritic with the PPO default networks, Buffer.finish_path) and utils/online_mean_std.py
(OnlineMeanStd) from /root/reference.  The mirror (cf2sim.rollout), the fused policy kernel
(cf2_policy_forward, observation standardisation in the kernel) and the GAE kernel (cf2_gae,
reward scaling, discounted returns) are checked against those outputs."""
import os

import numpy as np
import pytest
import torch

from cf2sim.rollout import MLPActorCritic, OnlineMeanStd, gae

G = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_f3.npz"))


def ref_ac(device="cpu"):
    ac = MLPActorCritic().to(device)
    ac.load_reference_state_dict({k[4:]: G[k] for k in G.files if k.startswith("ac__")})
    return ac.to(device)


def test_test_helper_discount_cumsum_matches_reference():
    from test_rollout import discount_cumsum
    np.testing.assert_allclose(discount_cumsum(G["dc_x"], 0.99), G["dc_099"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(discount_cumsum(G["dc_x"], 0.99 * 0.95), G["dc_09405"], rtol=1e-12, atol=1e-12)


def test_online_mean_std_matches_reference():
    oms = OnlineMeanStd(shape=(34,))
    for k in range(3):
        oms.update(torch.as_tensor(G[f"oms_batch{k}"]))
        np.testing.assert_allclose(oms.mean.numpy(), G[f"oms_mean{k}"], rtol=2e-6, atol=1e-6)
        np.testing.assert_allclose(oms.std.numpy(), G[f"oms_std{k}"], rtol=2e-6, atol=1e-6)
    probe = torch.as_tensor(G["oms_probe"])
    np.testing.assert_allclose(oms(probe).numpy(), G["oms_probe_out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(oms(probe, clip=True).numpy(), G["oms_probe_out_clip"], rtol=1e-5, atol=1e-5)
    with pytest.raises(ValueError):
        oms.update(torch.zeros(5, 33))


def test_actor_critic_matches_reference_outputs():
    ac = ref_ac()
    obs = torch.as_tensor(G["ac_obs"])
    mu, v, _ = ac.step(obs, deterministic=True)          # ac.eval(): predict() -> mu (core.py:284-290)
    np.testing.assert_allclose(mu.numpy(), G["ac_mu"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(v.numpy(), G["ac_v"], rtol=1e-5, atol=1e-6)
    lp = ac.log_prob(obs, torch.as_tensor(G["ac_acts"]))
    np.testing.assert_allclose(lp.numpy(), G["ac_logp"], rtol=1e-5, atol=1e-5)
    ac.set_log_std(0.3)
    # the reference's np.log(std) * float32 ones is float64 under numpy 2 promotion rules, float32
    # under numpy 1 (the reference's era); the mirror keeps the parameter float32
    np.testing.assert_allclose(ac.log_std.detach().numpy(), G["ac_log_std_frac03"], rtol=1e-7, atol=0)
    np.testing.assert_allclose(ac.log_prob(obs, torch.as_tensor(G["ac_acts"])).numpy(), G["ac_logp_frac03"],
                               rtol=1e-5, atol=1e-5)


def _episodes_as_buffer():
    """The golden episodes as one env's [T, 1] stream: each episode ends with done; a non-zero
    last_val is a cut-off (bootstrap V(s_T), here via trunc/trunc_val), zero a terminal state."""
    lens, last_vals = G["buf_lens"], G["buf_last_vals"]
    T = int(lens.sum())
    done = np.zeros(T, bool)
    trunc = np.zeros(T, bool)
    trunc_val = np.zeros(T, np.float32)
    t = 0
    for L, lv in zip(lens, last_vals):
        t += int(L)
        done[t - 1] = True
        trunc[t - 1] = lv != 0.0
        trunc_val[t - 1] = lv
    col = lambda x: x.reshape(T, 1)
    return col(G["buf_rew"]), col(G["buf_val"]), col(done), col(trunc), col(trunc_val)


@pytest.mark.parametrize("scaled", [False, True])
def test_batched_gae_matches_reference_finish_path(scaled):
    rew, val, done, trunc, trunc_val = (torch.as_tensor(x) for x in _episodes_as_buffer())
    den = float(G["buf_ret_std"][0]) + 1e-5 if scaled else None
    adv, tgt, disc = gae(rew.double(), val.double(), done, trunc, torch.zeros(1, dtype=torch.float64),
                         trunc_val.double(), 0.99, 0.95, rew_den=den, with_discounted=True)
    tag = "scaled" if scaled else "plain"
    np.testing.assert_allclose(adv[:, 0].numpy(), G[f"buf_adv_{tag}"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(tgt[:, 0].numpy(), G[f"buf_vtarget_{tag}"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(disc[:, 0].numpy(), G[f"buf_discret_{tag}"], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("scaled", [False, True])
def test_gae_kernel_matches_reference_finish_path(gpu, scaled):
    from cf2sim.rollout import gae_device
    rew, val, done, trunc, trunc_val = _episodes_as_buffer()
    g = lambda x: torch.as_tensor(x).to(gpu)
    den = float(G["buf_ret_std"][0]) + 1e-5 if scaled else None
    adv, tgt, disc = gae_device(g(rew), g(val), g(done.astype(np.uint8)), g(trunc.astype(np.uint8)),
                                torch.zeros(1, device=gpu), g(trunc_val), 0.99, 0.95, rew_den=den,
                                with_discounted=True)
    tag = "scaled" if scaled else "plain"
    np.testing.assert_allclose(adv[:, 0].cpu().numpy(), G[f"buf_adv_{tag}"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(tgt[:, 0].cpu().numpy(), G[f"buf_vtarget_{tag}"], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(disc[:, 0].cpu().numpy(), G[f"buf_discret_{tag}"], rtol=1e-5, atol=1e-4)


@pytest.mark.gpu
@pytest.mark.parametrize("precision,tol", [("fp32", 2e-5), ("bf16x3", 5e-5)])
def test_fused_policy_matches_reference_actor_critic(gpu, precision, tol):
    """The fused kernel with the reference's trained-shape weights and observation statistics
    (applied in the kernel) reproduces the reference's mu and V (fp32 products to 2e-5,
    split-bf16 products to 5e-5), and its log-probabilities equal the reference's
    Normal(mu, std).log_prob of the sampled actions."""
    from cf2sim.rollout import FusedActorCritic
    ac = ref_ac(gpu)
    fused = FusedActorCritic(ac, seed=3, precision=precision)
    obs = torch.as_tensor(G["ac_obs"]).to(gpu)
    mu, v, _ = fused.step(obs, deterministic=True)
    err = lambda a, b: float((np.abs(a - b) / (1 + np.abs(b))).max())
    print(f"{precision}: mu err {err(mu.cpu().numpy(), G['ac_mu']):.2e}, v err {err(v.cpu().numpy(), G['ac_v']):.2e}")
    assert err(mu.cpu().numpy(), G["ac_mu"]) < tol
    assert err(v.cpu().numpy(), G["ac_v"]) < tol
    a, _, lp = fused.step(obs)
    assert err(lp.cpu().numpy(), ac.log_prob(obs, a).cpu().numpy()) < 1e-4
