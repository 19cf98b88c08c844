"""Batched rollout caller: the reference's PPO/IWPG data collection
with every env of a GPU stepped at once instead of one env per MPI process.

Reference behaviour restated (paths relative to phoenix_drone_simulation/):

* ``ActorCritic`` (algs/core.py:300-395) with ``MLPGaussianActor`` (core.py:228-291) and
  ``MLPCritic``; PPO defaults (algs/ppo/defaults.py:8-17): pi 34->50->50->4 ReLU with a fixed
  log_std = log(0.5) (annealed by ``set_log_std``), v 34->64->64->1 tanh, gamma 0.99,
  lam 0.95 (algs/iwpg/iwpg.py:40), Linear layers, identity output.
* ``IWPGAlgorithm.roll_out`` (algs/iwpg/iwpg.py:372-410): step the policy, store
  (obs, act, rew, val, logp), and at an episode end call ``finish_path(last_val)`` with
  last_val = 0 on a terminal state and V(s) on a time-out or at the end of the epoch.
* ``finish_path`` / ``calculate_adv_and_value_targets`` (algs/core.py:459-535): GAE
  A_t = sum_k (gamma*lam)^k delta_{t+k}, delta_t = r_t + gamma V_{t+1} - V_t, value targets
  A_t + V_t, over each episode slice.

Here N envs run in lock step with on-device auto-reset, so episode boundaries differ per env.
``gae`` evaluates the same recursion over a [T, N] buffer with per-env masks:
terminal -> bootstrap 0; truncated (TimeLimit) -> bootstrap V(final_obs), the pre-reset
observation the env reports; end of the buffer -> V(obs_T).  This equals running the reference's
finish_path on every env's episode slices (tests/test_rollout.py checks exactly that).
One edge differs: roll_out tests its own ``ep_len == max_ep_len`` and so bootstraps a terminal
state reached exactly at the time limit; gym's TimeLimit (and this env) reports that step as
terminal, not truncated, and it bootstraps 0.
"""
from __future__ import annotations

import dataclasses
import math

import torch
from torch import nn


def _mlp(sizes, activation, output_activation=nn.Identity):
    layers = []
    for j in range(len(sizes) - 1):
        act = activation if j < len(sizes) - 2 else output_activation
        layers += [nn.Linear(sizes[j], sizes[j + 1]), act()]
    return nn.Sequential(*layers)


_ACT = {"relu": nn.ReLU, "tanh": nn.Tanh, "identity": nn.Identity}


class MLPActorCritic(nn.Module):
    """Gaussian MLP policy + MLP value function with the reference's PPO defaults."""

    def __init__(self, obs_dim: int = 34, act_dim: int = 4, pi_hidden=(50, 50), pi_activation="relu",
                 v_hidden=(64, 64), v_activation="tanh", log_std: float = math.log(0.5)):
        super().__init__()
        self.pi_net = _mlp([obs_dim, *pi_hidden, act_dim], _ACT[pi_activation])
        self.v_net = _mlp([obs_dim, *v_hidden, 1], _ACT[v_activation])
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std)), requires_grad=False)

    def set_log_std(self, frac: float):
        """Exploration-noise annealing of core.py:274-281 (std 0.5 -> 0.01 as frac goes 1 -> 0)."""
        assert 0.0 <= frac <= 1.0
        with torch.no_grad():
            self.log_std.fill_(math.log(0.499 * frac + 0.01))

    @torch.no_grad()
    def step(self, obs: torch.Tensor, generator: torch.Generator | None = None, deterministic: bool = False):
        """(action, value, log_prob) for a batch of observations (core.py:371-395)."""
        mu = self.pi_net(obs)
        v = self.v_net(obs).squeeze(-1)
        if deterministic:
            return mu, v, torch.ones_like(mu)
        std = self.log_std.exp()
        eps = torch.randn(mu.shape, device=mu.device, dtype=mu.dtype, generator=generator)
        a = mu + std * eps
        # Normal(mu, std).log_prob(a).sum(-1)
        logp = (-0.5 * eps.pow(2) - self.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
        return a, v, logp

    @torch.no_grad()
    def value(self, obs: torch.Tensor) -> torch.Tensor:
        return self.v_net(obs).squeeze(-1)


def pack_policy_weights(ac: MLPActorCritic) -> torch.Tensor:
    """Flatten an MLPActorCritic with the default shapes into the weight block of
    cf2_policy_forward (input-major matrices: pi W1 b1 W2 b2 W3 b3 log_std, then v W1 b1 W2 b2 W3 b3)."""
    lin_pi = [m for m in ac.pi_net if isinstance(m, nn.Linear)]
    lin_v = [m for m in ac.v_net if isinstance(m, nn.Linear)]
    shapes = [(m.out_features, m.in_features) for m in lin_pi] + [(m.out_features, m.in_features) for m in lin_v]
    d = lin_pi[0].in_features
    if shapes != [(50, d), (50, 50), (4, 50), (64, d), (64, 64), (1, 64)] or d not in (34, 42):
        raise ValueError(f"the fused kernel implements the PPO default networks only, got {shapes}")
    parts = []
    for m in lin_pi:
        parts += [m.weight.detach().t().reshape(-1), m.bias.detach()]
    parts.append(ac.log_std.detach())
    for m in lin_v:
        parts += [m.weight.detach().t().reshape(-1), m.bias.detach()]
    return torch.cat([p.float().reshape(-1) for p in parts]).contiguous()


class FusedActorCritic:
    """``MLPActorCritic.step`` / ``value`` through the fused HIP kernel (cf2_policy_forward).
    Sampling noise comes from Philox keyed (seed, call counter, row): reproducible, independent
    of batch geometry.  Call ``sync()`` after changing the torch module's parameters."""

    def __init__(self, ac: MLPActorCritic, seed: int = 0):
        from . import _native
        self.ac = ac
        self.lib = _native.load()
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.counter = 0
        self.obs_dim = ac.pi_net[0].in_features
        self.sync()

    def sync(self):
        dev = next(self.ac.parameters()).device
        self.w = pack_policy_weights(self.ac).to(dev)
        assert self.w.numel() == self.lib.cf2_policy_weights_count(self.obs_dim)

    @torch.no_grad()
    def step(self, obs: torch.Tensor, deterministic: bool = False, row_offset: int = 0):
        from . import _native
        n = obs.shape[0]
        obs = obs.contiguous()
        act = torch.empty(n, 4, device=obs.device)
        val = torch.empty(n, device=obs.device)
        logp = torch.empty(n, device=obs.device)
        _native.check(self.lib.cf2_policy_forward(
            self.w.data_ptr(), n, self.obs_dim, obs.data_ptr(), self.seed, self.counter & 0xFFFFFFFF, row_offset,
            0 if deterministic else 1, act.data_ptr(), val.data_ptr(), logp.data_ptr(),
            torch.cuda.current_stream(obs.device).cuda_stream), "cf2_policy_forward")
        self.counter += 1
        return act, val, logp

    @torch.no_grad()
    def step_into(self, obs: torch.Tensor, act: torch.Tensor, val: torch.Tensor, logp: torch.Tensor):
        from . import _native
        _native.check(self.lib.cf2_policy_forward(
            self.w.data_ptr(), obs.shape[0], self.obs_dim, obs.data_ptr(), self.seed, self.counter & 0xFFFFFFFF, 0, 1,
            act.data_ptr(), val.data_ptr(), logp.data_ptr(), torch.cuda.current_stream(obs.device).cuda_stream),
            "cf2_policy_forward")
        self.counter += 1

    @torch.no_grad()
    def value_masked(self, obs: torch.Tensor, mask: torch.Tensor, out: torch.Tensor):
        from . import _native
        _native.check(self.lib.cf2_value_forward_masked(
            self.w.data_ptr(), obs.shape[0], self.obs_dim, obs.contiguous().data_ptr(),
            mask.to(torch.uint8).contiguous().data_ptr(), out.data_ptr(),
            torch.cuda.current_stream(obs.device).cuda_stream), "cf2_value_forward_masked")
        return out

    @torch.no_grad()
    def value(self, obs: torch.Tensor) -> torch.Tensor:
        return self.step(obs, deterministic=True)[1]


def gae(rew, val, done, trunc, last_val, trunc_val, gamma: float = 0.99, lam: float = 0.95):
    """Batched GAE over [T, N] buffers with per-env episode boundaries.

    rew, val:   [T, N] rewards r_t and values V(s_t)
    done:       [T, N] bool, episode ended at t (terminal or truncated; the env auto-reset)
    trunc:      [T, N] bool, the end was a TimeLimit truncation (bootstrap from trunc_val)
    last_val:   [N]    V(s_T) of the observation after the last step (epoch cut-off)
    trunc_val:  [T, N] V(final_obs_t) where trunc, anything elsewhere
    Returns (adv [T, N], value_targets [T, N])."""
    T = rew.shape[0]
    adv = torch.empty_like(rew)
    nxt_adv = torch.zeros_like(last_val)
    nxt_val = last_val
    for t in range(T - 1, -1, -1):
        d = done[t]
        boot = torch.where(d, torch.where(trunc[t], trunc_val[t], torch.zeros_like(nxt_val)), nxt_val)
        delta = rew[t] + gamma * boot - val[t]
        a = delta + gamma * lam * torch.where(d, torch.zeros_like(nxt_adv), nxt_adv)
        adv[t] = a
        nxt_adv, nxt_val = a, val[t]
    return adv, adv + val


def gae_device(rew, val, done_u8, trunc_u8, last_val, trunc_val, gamma: float = 0.99, lam: float = 0.95):
    """``gae`` as one HIP launch (cf2_gae): one thread per env scans T backward."""
    from . import _native
    T, n = rew.shape
    adv = torch.empty_like(rew)
    ret = torch.empty_like(rew)
    lib = _native.load()
    _native.check(lib.cf2_gae(T, n, rew.contiguous().data_ptr(), val.contiguous().data_ptr(),
                              done_u8.contiguous().data_ptr(), trunc_u8.contiguous().data_ptr(),
                              trunc_val.contiguous().data_ptr(), last_val.contiguous().data_ptr(), float(gamma),
                              float(lam), adv.data_ptr(), ret.data_ptr(),
                              torch.cuda.current_stream(rew.device).cuda_stream), "cf2_gae")
    return adv, ret


@dataclasses.dataclass
class Rollout:
    obs: torch.Tensor        # [T, N, obs_dim]
    act: torch.Tensor        # [T, N, 4]
    rew: torch.Tensor        # [T, N]
    val: torch.Tensor        # [T, N]
    logp: torch.Tensor       # [T, N]
    done: torch.Tensor       # [T, N] bool
    trunc: torch.Tensor      # [T, N] bool
    adv: torch.Tensor        # [T, N]
    ret: torch.Tensor        # [T, N] value-function targets
    last_obs: torch.Tensor   # [N, obs_dim] observation after the last step
    last_val: torch.Tensor   # [N] V(last_obs)
    trunc_val: torch.Tensor  # [T, N] V(pre-reset obs), used where trunc


@torch.no_grad()
def collect(envs, ac, steps: int, obs: torch.Tensor | None = None, gamma: float = 0.99,
            lam: float = 0.95, generator: torch.Generator | None = None) -> Rollout:
    """``roll_out`` for all envs of a BatchedCrazyflieEnv at once; everything stays on the GPU.
    ``ac`` is an MLPActorCritic (torch layers) or a FusedActorCritic (one HIP launch per step).
    ``envs`` must have been created with want_final_obs=True (time-out bootstrapping)."""
    if envs.final_obs is None:
        raise ValueError("collect() needs BatchedCrazyflieEnv(..., want_final_obs=True)")
    n, d, dev = envs.num_envs, envs.obs_dim, envs.device
    o = envs.reset() if obs is None else obs
    buf_o = torch.empty(steps, n, d, device=dev)
    buf_a = torch.empty(steps, n, 4, device=dev)
    buf_r = torch.empty(steps, n, device=dev)
    buf_v = torch.empty(steps, n, device=dev)
    buf_lp = torch.empty(steps, n, device=dev)
    buf_d = torch.empty(steps, n, dtype=torch.bool, device=dev)
    buf_tr = torch.empty(steps, n, dtype=torch.bool, device=dev)
    trunc_val = torch.zeros(steps, n, device=dev)
    fused = isinstance(ac, FusedActorCritic)
    if fused:
        # zero-copy: the policy and the env write straight into the rollout storage
        obs_buf = torch.empty(steps + 1, n, d, device=dev)
        obs_buf[0] = o
        d8 = torch.empty(steps, n, dtype=torch.uint8, device=dev)
        tr8 = torch.empty(steps, n, dtype=torch.uint8, device=dev)
        fin = envs.final_obs
        for t in range(steps):
            ac.step_into(obs_buf[t], buf_a[t], buf_v[t], buf_lp[t])
            envs.step_into(buf_a[t], obs_buf[t + 1], buf_r[t], d8[t], tr8[t], final_obs_out=fin)
            ac.value_masked(fin, tr8[t], trunc_val[t])              # V(final obs) of the time-outs only
        o = obs_buf[steps]
        last_val = ac.value(o)
        adv, ret = gae_device(buf_r, buf_v, d8, tr8, last_val, trunc_val, gamma, lam)
        buf_o, buf_d, buf_tr = obs_buf[:steps], d8.bool(), tr8.bool()
        return Rollout(buf_o, buf_a, buf_r, buf_v, buf_lp, buf_d, buf_tr, adv, ret, o, last_val, trunc_val)
    for t in range(steps):
        a, v, lp = ac.step(o, generator=generator)
        buf_o[t] = o
        buf_a[t] = a
        buf_v[t] = v
        buf_lp[t] = lp
        o, r, dn, info = envs.step(a.contiguous())
        buf_r[t] = r
        buf_d[t] = dn.bool()
        buf_tr[t] = info["truncated"].bool()
        trunc_val[t] = ac.value(info["final_obs"])      # only read where truncated
    last_val = ac.value(o)
    adv, ret = gae(buf_r, buf_v, buf_d, buf_tr, last_val, trunc_val, gamma, lam)
    return Rollout(buf_o, buf_a, buf_r, buf_v, buf_lp, buf_d, buf_tr, adv, ret, o, last_val, trunc_val)


__all__ = ["MLPActorCritic", "FusedActorCritic", "pack_policy_weights", "gae", "gae_device", "collect", "Rollout"]
