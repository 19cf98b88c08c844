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
  A_t + V_t, over each episode slice; with reward scaling (IWPG default use_reward_scaling=True,
  algs/iwpg/iwpg.py:56) the rewards entering delta are clip(r / (ret_std + 1e-5), -10, 10)
  (core.py:522-529) and the unscaled discounted returns feed the return statistics.
* Observation standardisation (IWPG default use_standardized_obs=True, iwpg.py:59):
  ``ActorCritic.step`` feeds (obs - mean) / (std + 1e-5) to both networks (core.py:383-388);
  the statistics are ``OnlineMeanStd`` (utils/online_mean_std.py), updated once per epoch by
  ``update_running_statistics`` (iwpg.py:412-420).  The fused kernel standardises the observation
  in registers before the first layer (pack_policy_weights carries mean and 1 / (std + eps)).

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


class OnlineMeanStd(nn.Module):
    """Running mean / standard deviation (utils/online_mean_std.py): the incremental update of
    Chan et al. over batches, single process (the reference's MPI averages are the identity with
    one process; across GPUs, batches of every rank can be concatenated before update()).

    Provenance: this restates the reference's OnlineMeanStd closely -- same epsilon, same clip
    bound 10, the same n_A / n_AB / delta / mean / M2 update in the same order -- because the
    standardised observations must reproduce the reference's arithmetic to match
    tests/golden/golden_f3.npz (generated from the reference's own class).  It is a ~35-line
    standard algorithm, not new design."""

    def __init__(self, epsilon: float = 1e-5, shape=()):
        super().__init__()
        self.register_buffer("mean", torch.zeros(*shape))
        self.register_buffer("std", torch.ones(*shape))
        self.register_buffer("count", torch.zeros(1))
        self.eps = epsilon
        self.bound = 10
        self.shape = tuple(shape)

    def forward(self, x, subtract_mean: bool = True, clip: bool = False):
        x_new = (x - self.mean) / (self.std + self.eps) if subtract_mean else x / (self.std + self.eps)
        return torch.clamp(x_new, -self.bound, self.bound) if clip else x_new

    def std_host(self) -> float:
        """std as a host float (shape (1,) statistics), re-read from the device only after the
        buffer changed (in place or replaced): collect() needs it every epoch for reward scaling,
        and a device read would drain the GPU's queue at the start of every collect."""
        t = self.std
        if getattr(self, "_std_host_key", None) is None or self._std_host_key[0] is not t \
                or self._std_host_key[1] != t._version:
            self._std_host = float(t.item())
            self._std_host_key = (t, t._version)
        return self._std_host

    @torch.no_grad()
    def update(self, x: torch.Tensor) -> None:
        x = torch.as_tensor(x, dtype=torch.float32, device=self.mean.device)
        if self.shape[0] == 1:
            if x.dim() != 1:
                raise ValueError(f"expected a 1-d batch, got {tuple(x.shape)}")
            x = x.view(-1, 1)
        elif x.dim() != 2 or x.shape[1] != self.shape[0]:
            raise ValueError(f"expected [B, {self.shape[0]}], got {tuple(x.shape)}")
        n_b = x.shape[0]
        n_a = self.count.clone()
        n_ab = self.count + n_b
        delta = x.mean(dim=0) - self.mean
        mean_new = self.mean + delta * n_b / n_ab
        batch_var = torch.mean((x - mean_new) ** 2, dim=0)
        m2_ab = n_a * torch.square(self.std) + n_b * batch_var + delta ** 2 * (n_a * n_b / n_ab)
        self.mean.copy_(mean_new)
        self.count.copy_(n_ab)
        self.std.copy_(torch.sqrt(m2_ab / n_ab))


class MLPActorCritic(nn.Module):
    """Gaussian MLP policy + MLP value function with the reference's PPO defaults, the
    observation standardisation and the return statistics of reward scaling."""

    def __init__(self, obs_dim: int = 34, act_dim: int = 4, pi_hidden=(50, 50), pi_activation="relu",
                 v_hidden=(64, 64), v_activation="tanh", log_std: float = math.log(0.5),
                 use_standardized_obs: bool = True, use_scaled_rewards: bool = True):
        super().__init__()
        self.pi_net = _mlp([obs_dim, *pi_hidden, act_dim], _ACT[pi_activation])
        self.v_net = _mlp([obs_dim, *v_hidden, 1], _ACT[v_activation])
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std)), requires_grad=False)
        self.obs_oms = OnlineMeanStd(shape=(obs_dim,)) if use_standardized_obs else None
        self.ret_oms = OnlineMeanStd(shape=(1,)) if use_scaled_rewards else None

    def load_reference_state_dict(self, sd: dict):
        """Load a state_dict of the reference's ActorCritic (keys pi.net.{0,2,4}.*, pi.log_std,
        v.net.{0,2,4}.*, obs_oms.*, ret_oms.*; algs/core.py:314-364)."""
        def t(k):
            return torch.as_tensor(sd[k], dtype=torch.float32)
        with torch.no_grad():
            for mine, ref in ((self.pi_net, "pi.net"), (self.v_net, "v.net")):
                for i in (0, 2, 4):
                    mine[i].weight.copy_(t(f"{ref}.{i}.weight"))
                    mine[i].bias.copy_(t(f"{ref}.{i}.bias"))
            self.log_std.copy_(t("pi.log_std"))
            for name, oms in (("obs_oms", self.obs_oms), ("ret_oms", self.ret_oms)):
                if oms is not None and f"{name}.mean" in sd:
                    oms.mean.copy_(t(f"{name}.mean")); oms.std.copy_(t(f"{name}.std")); oms.count.copy_(t(f"{name}.count"))

    def normalize(self, obs: torch.Tensor) -> torch.Tensor:
        return self.obs_oms(obs) if self.obs_oms is not None else obs

    def set_log_std(self, frac: float):
        """Exploration-noise annealing of core.py:274-281 (std 0.5 -> 0.01 as frac goes 1 -> 0)."""
        assert 0.0 <= frac <= 1.0
        with torch.no_grad():
            self.log_std.fill_(math.log(0.499 * frac + 0.01))

    @torch.no_grad()
    def step(self, obs: torch.Tensor, generator: torch.Generator | None = None, deterministic: bool = False):
        """(action, value, log_prob) for a batch of observations (core.py:371-395)."""
        obs = self.normalize(obs)
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
        return self.v_net(self.normalize(obs)).squeeze(-1)

    @torch.no_grad()
    def log_prob(self, obs: torch.Tensor, act: torch.Tensor) -> torch.Tensor:
        """Normal(mu(obs), std).log_prob(act).sum(-1) (core.py:253-259)."""
        mu = self.pi_net(self.normalize(obs))
        return torch.distributions.Normal(mu, self.log_std.exp()).log_prob(act).sum(-1)


def update_running_statistics(ac: MLPActorCritic, rollout: "Rollout", fused: "FusedActorCritic | None" = None):
    """IWPGAlgorithm.update_running_statistics (iwpg.py:412-420) on a whole batched rollout: the raw
    observations update the observation statistics, the discounted returns the return statistics.
    A FusedActorCritic over `ac` is re-synced (its weight block carries the standardisation)."""
    if ac.obs_oms is not None:
        ac.obs_oms.update(rollout.obs.reshape(-1, rollout.obs.shape[-1]))
    if ac.ret_oms is not None:
        ac.ret_oms.update(rollout.discounted_ret.reshape(-1))
    if fused is not None:
        fused.sync()


def pack_policy_weights(ac: MLPActorCritic) -> torch.Tensor:
    """Flatten an MLPActorCritic with the default shapes into the flat weight block of
    cf2_policy_pack (input-major matrices: pi W1 b1 W2 b2 W3 b3 log_std, then v W1 b1 W2 b2 W3 b3,
    then the observation standardisation mean[D] and scale[D] = 1 / (std + eps), computed in fp64;
    identity without obs_oms).  The kernel standardises the observation before the first layer,
    as ActorCritic.step does (core.py:383-388)."""
    lin_pi = [m for m in ac.pi_net if isinstance(m, nn.Linear)]
    lin_v = [m for m in ac.v_net if isinstance(m, nn.Linear)]
    shapes = [(m.out_features, m.in_features) for m in lin_pi] + [(m.out_features, m.in_features) for m in lin_v]
    d = lin_pi[0].in_features
    if shapes != [(50, d), (50, 50), (4, 50), (64, d), (64, 64), (1, 64)] or d not in (34, 42):
        raise ValueError(f"the fused kernel implements the PPO default networks only, got {shapes}")
    parts = []
    for lins in (lin_pi, lin_v):
        for m in lins:
            parts += [m.weight.detach().t().reshape(-1), m.bias.detach()]
        if lins is lin_pi:
            parts.append(ac.log_std.detach())
    dev = lin_pi[0].weight.device
    if ac.obs_oms is not None:
        parts += [ac.obs_oms.mean.detach(), 1.0 / (ac.obs_oms.std.detach().double() + ac.obs_oms.eps)]
    else:
        parts += [torch.zeros(d, device=dev), torch.ones(d, device=dev)]
    return torch.cat([p.float().reshape(-1) for p in parts]).contiguous()


POLICY_PRECISIONS = {"fp32": 0, "bf16x3": 1}     # cf2_policy_precision (include/cf2sim.h)


class FusedActorCritic:
    """``MLPActorCritic.step`` / ``value`` through the fused HIP kernel (cf2_policy_forward).
    Sampling noise comes from Philox keyed (seed, call counter, row): reproducible, independent
    of batch geometry.  Call ``sync()`` after changing the torch module's parameters.

    precision: "fp32" -- exact fp32 products on the matrix cores (the result of an fmaf chain);
    "bf16x3" -- split-bf16 products (x = hi + lo, three bf16 MFMAs): <= ~1.1e-5 relative error
    per product, fp32 accumulation and activations, ~5x the fp32 matrix rate.  The collected
    log-probabilities do not depend on it (logp is a function of the drawn noise only)."""

    def __init__(self, ac: MLPActorCritic, seed: int = 0, precision: str = "bf16x3"):
        from . import _native
        if precision not in POLICY_PRECISIONS:
            raise ValueError(f"precision must be one of {sorted(POLICY_PRECISIONS)}, got {precision!r}")
        self.ac = ac
        self.lib = _native.load()
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        self.counter = 0
        self.precision = precision
        self.prec = POLICY_PRECISIONS[precision]
        self.obs_dim = ac.pi_net[0].in_features
        self.sync()

    def sync(self):
        """Re-pack the weights: the flat block (pack_policy_weights) -> the kernel's MFMA fragment
        block (cf2_policy_pack, one launch)."""
        from . import _native
        dev = next(self.ac.parameters()).device
        flat = pack_policy_weights(self.ac).to(dev)
        assert flat.numel() == self.lib.cf2_policy_weights_count(self.obs_dim)
        self.w = torch.empty(self.lib.cf2_policy_packed_count(self.obs_dim, self.prec), device=dev)
        self.w_ptr = self.w.data_ptr()
        _native.check(self.lib.cf2_policy_pack(flat.data_ptr(), self.obs_dim, self.prec, self.w.data_ptr(),
                                               torch.cuda.current_stream(dev).cuda_stream), "cf2_policy_pack")

    @torch.no_grad()
    def step(self, obs: torch.Tensor, deterministic: bool = False, row_offset: int = 0):
        from . import _native
        n = obs.shape[0]
        obs = obs.contiguous()
        act = torch.empty(n, 4, device=obs.device)
        val = torch.empty(n, device=obs.device)
        logp = torch.empty(n, device=obs.device)
        _native.check(self.lib.cf2_policy_forward(
            self.w.data_ptr(), n, self.obs_dim, self.prec, obs.data_ptr(), self.seed, self.counter & 0xFFFFFFFF, row_offset,
            0 if deterministic else 1, act.data_ptr(), val.data_ptr(), logp.data_ptr(),
            torch.cuda.current_stream(obs.device).cuda_stream), "cf2_policy_forward")
        self.counter += 1
        return act, val, logp

    @torch.no_grad()
    def step_into(self, obs: torch.Tensor, act: torch.Tensor, val: torch.Tensor, logp: torch.Tensor,
                  row_offset: int = 0):
        """step() into caller buffers.  row_offset: global index of row 0 (the sampling noise of row
        r is keyed by row_offset + r; collect() passes the env shard's env_id_offset, so a rank's
        envs draw the noise they would draw in one process holding every env)."""
        from . import _native
        _native.check(self.lib.cf2_policy_forward(
            self.w.data_ptr(), obs.shape[0], self.obs_dim, self.prec, obs.data_ptr(), self.seed,
            self.counter & 0xFFFFFFFF, int(row_offset), 1,
            act.data_ptr(), val.data_ptr(), logp.data_ptr(), torch.cuda.current_stream(obs.device).cuda_stream),
            "cf2_policy_forward")
        self.counter += 1

    @torch.no_grad()
    def value_masked(self, obs: torch.Tensor, mask: torch.Tensor, out: torch.Tensor):
        from . import _native
        _native.check(self.lib.cf2_value_forward_masked(
            self.w.data_ptr(), obs.shape[0], self.obs_dim, self.prec, obs.contiguous().data_ptr(),
            mask.to(torch.uint8).contiguous().data_ptr(), out.data_ptr(),
            torch.cuda.current_stream(obs.device).cuda_stream), "cf2_value_forward_masked")
        return out

    @torch.no_grad()
    def value(self, obs: torch.Tensor) -> torch.Tensor:
        return self.step(obs, deterministic=True)[1]


def gae(rew, val, done, trunc, last_val, trunc_val, gamma: float = 0.99, lam: float = 0.95,
        rew_den: float | None = None, with_discounted: bool = False):
    """Batched GAE over [T, N] buffers with per-env episode boundaries.

    rew, val:   [T, N] rewards r_t and values V(s_t)
    done:       [T, N] bool, episode ended at t (terminal or truncated; the env auto-reset)
    trunc:      [T, N] bool, the end was a TimeLimit truncation (bootstrap from trunc_val)
    last_val:   [N]    V(s_T) of the observation after the last step (epoch cut-off)
    trunc_val:  [T, N] V(final_obs_t) where trunc, anything elsewhere
    rew_den:    reward scaling (core.py:522-529): delta uses clip(r / rew_den, -10, 10) with
                rew_den = ret_oms.std + 1e-5; None = unscaled
    Returns (adv [T, N], value_targets [T, N]) and, with with_discounted, the per-episode
    discounted returns of the unscaled rewards bootstrapped like finish_path (core.py:519)."""
    T = rew.shape[0]
    adv = torch.empty_like(rew)
    disc = torch.empty_like(rew) if with_discounted else None
    nxt_adv = torch.zeros_like(last_val)
    nxt_val = last_val
    nxt_ret = last_val
    for t in range(T - 1, -1, -1):
        d = done[t]
        boot = torch.where(d, torch.where(trunc[t], trunc_val[t], torch.zeros_like(nxt_val)), nxt_val)
        r = rew[t] if rew_den is None else torch.clamp(rew[t] / rew_den, -10.0, 10.0)
        delta = r + gamma * boot - val[t]
        a = delta + gamma * lam * torch.where(d, torch.zeros_like(nxt_adv), nxt_adv)
        adv[t] = a
        if disc is not None:
            disc[t] = rew[t] + gamma * torch.where(d, boot, nxt_ret)
            nxt_ret = disc[t]
        nxt_adv, nxt_val = a, val[t]
    return (adv, adv + val, disc) if with_discounted else (adv, adv + val)


def gae_device(rew, val, done_u8, trunc_u8, last_val, trunc_val, gamma: float = 0.99, lam: float = 0.95,
               rew_den: float | None = None, with_discounted: bool = False, out=None):
    """``gae`` as one HIP launch (cf2_gae): one thread per env scans T backward.  out: optional
    (adv, ret, disc) [T, N] float32 buffers to write."""
    from . import _native
    T, n = rew.shape
    if out is not None:
        adv, ret, disc = out
        for b in (adv, ret) + ((disc,) if with_discounted else ()):
            if b.shape != rew.shape or b.dtype != torch.float32 or not b.is_contiguous() or b.device != rew.device:
                raise ValueError("gae_device out buffers must be contiguous float32 [T, N] on the same device")
        disc = disc if with_discounted else None
    else:
        adv = torch.empty_like(rew)
        ret = torch.empty_like(rew)
        disc = torch.empty_like(rew) if with_discounted else None
    lib = _native.load()
    _native.check(lib.cf2_gae(T, n, rew.contiguous().data_ptr(), val.contiguous().data_ptr(),
                              done_u8.contiguous().data_ptr(), trunc_u8.contiguous().data_ptr(),
                              trunc_val.contiguous().data_ptr(), last_val.contiguous().data_ptr(), float(gamma),
                              float(lam), float(rew_den) if rew_den is not None else 0.0, adv.data_ptr(),
                              ret.data_ptr(), _native.ptr(disc), torch.cuda.current_stream(rew.device).cuda_stream),
                  "cf2_gae")
    return (adv, ret, disc) if with_discounted else (adv, ret)


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
    discounted_ret: torch.Tensor  # [T, N] per-episode discounted returns (return statistics)
    # the fused path's buffers, re-used by collect(..., out=this rollout)
    storage: dict | None = dataclasses.field(default=None, repr=False, compare=False)


def _fused_storage(steps: int, n: int, d: int, dev) -> dict:
    """The fused collect path's rollout storage: observations [T+1, N, D] (slab 0 = the start
    observation), final observations [T, N, D] (rows written where an episode ended), actions,
    values and log-probabilities [T+1, ...] (slab T: the policy call on the last observation),
    rewards, uint8 done / truncation flags and the GAE outputs."""
    e = lambda *shape, dt=torch.float32: torch.empty(*shape, device=dev, dtype=dt)
    return {"key": (steps, n, d, str(dev)), "obs": e(steps + 1, n, d), "fin": e(steps, n, d),
            "act": e(steps + 1, n, 4), "rew": e(steps, n), "val": e(steps + 1, n), "logp": e(steps + 1, n),
            "d8": e(steps, n, dt=torch.uint8), "tr8": e(steps, n, dt=torch.uint8), "trunc_val": e(steps, n),
            "adv": e(steps, n), "ret": e(steps, n), "disc": e(steps, n)}


@torch.no_grad()
def collect(envs, ac, steps: int, obs: torch.Tensor | None = None, gamma: float = 0.99,
            lam: float = 0.95, generator: torch.Generator | None = None, fuse: bool | str = True,
            out: Rollout | None = None) -> Rollout:
    """``roll_out`` for all envs of a BatchedCrazyflieEnv at once; everything stays on the GPU.
    ``ac`` is an MLPActorCritic (torch layers) or a FusedActorCritic (HIP kernels).  With a
    FusedActorCritic, ``fuse`` picks how the loop's env-steps and policy calls are launched where
    the config has fused instances: True -- all ``steps`` of them in one launch
    (cf2_collect_rollout, the env state in registers throughout); "steps" -- one launch per
    env-step (cf2_collect_step); False -- two launches per env-step.  The results are
    bit-identical in every mode, and a config without fused instances runs the two launches.
    ``out``: a Rollout of an earlier fused collect of the
    same shape whose storage is re-used (its tensors are overwritten; ``obs=out.last_obs`` is
    allowed), as a training loop collecting every epoch would.
    ``envs`` must have been created with want_final_obs=True (time-out bootstrapping)."""
    if envs.final_obs is None:
        raise ValueError("collect() needs BatchedCrazyflieEnv(..., want_final_obs=True)")
    n, d, dev = envs.num_envs, envs.obs_dim, envs.device
    o = envs.reset() if obs is None else obs
    fused = isinstance(ac, FusedActorCritic)
    module = ac.ac if fused else ac
    rew_den = module.ret_oms.std_host() + module.ret_oms.eps if module.ret_oms is not None else None
    if fused:
        # zero-copy: the policy and the env write straight into the rollout storage
        S = out.storage if out is not None and out.storage is not None else None
        if S is None or S["key"] != (steps, n, d, str(dev)):
            S = _fused_storage(steps, n, d, dev)
        obs_buf, fin, act_all, buf_r, val_all, lp_all = S["obs"], S["fin"], S["act"], S["rew"], S["val"], S["logp"]
        buf_a, buf_v, buf_lp, last_val = act_all[:steps], val_all[:steps], lp_all[:steps], val_all[steps]
        d8, tr8, trunc_val = S["d8"], S["tr8"], S["trunc_val"]
        obs_buf[0].copy_(o)
        trunc_val.zero_()                 # read only where truncated; zero elsewhere, as the torch path
        # the policy of step t + 1 runs right behind the env-step of step t (fused: in its launch);
        # the last one gives V(obs_T), its sampled action and logp are not used
        roff = int(envs.cfg.env_id_offset)    # sampling noise keyed by the global env id
        ac.step_into(obs_buf[0], act_all[0], val_all[0], lp_all[0], row_offset=roff)
        if fuse is True and not envs.collect_rollout_into(act_all, obs_buf[1:], buf_r, d8, tr8, fin, ac, val_all,
                                                          lp_all):
            fuse = False                       # no fused instance for this config: two launches per step
        for t in range(steps if fuse is True else 0, steps):
            nxt = (act_all[t + 1], val_all[t + 1], lp_all[t + 1])
            if fuse and t == 0:
                # the first step goes through every buffer check; the later slabs have the same
                # shapes, so the loop then passes raw pointers (slab strides) to keep ahead of the GPU
                if envs.collect_step_into(buf_a[0], obs_buf[1], buf_r[0], d8[0], tr8[0], fin[0], ac, *nxt):
                    continue
                fuse = False
            elif fuse:
                sa, so, sf = n * 16, n * d * 4, n * 4            # slab strides in bytes
                a_p, o_p, r_p, v_p, l_p, f_p = (buf_a.data_ptr(), obs_buf.data_ptr(), buf_r.data_ptr(),
                                                buf_v.data_ptr(), buf_lp.data_ptr(), fin.data_ptr())
                dp, tp = d8.data_ptr(), tr8.data_ptr()
                for u in range(t, steps):
                    nx = (a_p + (u + 1) * sa, v_p + (u + 1) * sf, l_p + (u + 1) * sf)
                    if not envs.collect_step_raw(a_p + u * sa, o_p + (u + 1) * so, r_p + u * sf, dp + u * n, tp + u * n,
                                                 f_p + u * so, ac, *nx):
                        raise RuntimeError("cf2_collect_step stopped being supported inside a collect")
                envs._obs_latest = obs_buf[steps]    # what save_checkpoint saves after this collect
                break
            envs.step_into(buf_a[t], obs_buf[t + 1], buf_r[t], d8[t], tr8[t], final_obs_out=fin[t])
            ac.step_into(obs_buf[t + 1], *nxt, row_offset=roff)
        per = max(1, (2**31 - 1) // n)                      # row counts of the C ABI are 32-bit
        for t0 in range(0, steps, per):                      # V(final obs) of the time-outs only
            t1 = min(steps, t0 + per)
            ac.value_masked(fin[t0:t1].view(-1, d), tr8[t0:t1].view(-1), trunc_val[t0:t1].view(-1))
        envs.last_collect_fused = fuse         # True / "steps": every env-step ran fused (the mode that ran)
        o = obs_buf[steps]
        adv, ret, disc = gae_device(buf_r, buf_v, d8, tr8, last_val, trunc_val, gamma, lam, rew_den, True,
                                    out=(S["adv"], S["ret"], S["disc"]))
        buf_o, buf_d, buf_tr = obs_buf[:steps], d8.view(torch.bool), tr8.view(torch.bool)   # 0/1 bytes
        return Rollout(buf_o, buf_a, buf_r, buf_v, buf_lp, buf_d, buf_tr, adv, ret, o, last_val, trunc_val, disc,
                       storage=S)
    buf_o = torch.empty(steps, n, d, device=dev)
    buf_a = torch.empty(steps, n, 4, device=dev)
    buf_r = torch.empty(steps, n, device=dev)
    buf_v = torch.empty(steps, n, device=dev)
    buf_lp = torch.empty(steps, n, device=dev)
    buf_d = torch.empty(steps, n, dtype=torch.bool, device=dev)
    buf_tr = torch.empty(steps, n, dtype=torch.bool, device=dev)
    trunc_val = torch.zeros(steps, n, device=dev)
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
    adv, ret, disc = gae(buf_r, buf_v, buf_d, buf_tr, last_val, trunc_val, gamma, lam, rew_den, True)
    return Rollout(buf_o, buf_a, buf_r, buf_v, buf_lp, buf_d, buf_tr, adv, ret, o, last_val, trunc_val, disc)


__all__ = ["OnlineMeanStd", "MLPActorCritic", "FusedActorCritic", "pack_policy_weights", "gae", "gae_device", "collect",
           "Rollout", "update_running_statistics"]
