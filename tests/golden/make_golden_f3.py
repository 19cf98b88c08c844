"""Golden vectors of the rollout caller from the REFERENCE's own
learner code: phoenix_drone_simulation/algs/core.py (discount_cumsum, ActorCritic with the PPO
default networks, Buffer.finish_path with reward scaling) and utils/online_mean_std.py
(OnlineMeanStd), imported from /root/reference in this container with the stand-ins of
make_golden.py plus a one-process mpi4py stand-in (COMM_WORLD of size 1: every MPI average is the
identity, exactly the single-process path of the reference).  Run once where /root/reference
exists; writes tests/golden/golden_f3.npz (data only).  The tests never read the reference.
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402


def install_f3_stubs():
    make_golden.install_stubs()
    gym = sys.modules["gym"]

    class Discrete:  # noqa: E306
        def __init__(self, n):
            self.n = n
    gym.spaces.Discrete = Discrete
    mpi = types.ModuleType("mpi4py")

    class _Comm:  # noqa: E306
        def Get_size(self):
            return 1

        def Get_rank(self):
            return 0
    mpi.MPI = types.SimpleNamespace(COMM_WORLD=_Comm(), SUM="sum", MAX="max", MIN="min")
    sys.modules["mpi4py"] = mpi


def main():
    install_f3_stubs()
    import torch
    from phoenix_drone_simulation.algs import core
    from phoenix_drone_simulation.algs.ppo.defaults import defaults
    from phoenix_drone_simulation.utils.online_mean_std import OnlineMeanStd

    rec = {}
    rng = np.random.default_rng(2024)
    # ---- discount_cumsum (core.py:105-119)
    x = rng.normal(size=41)
    rec["dc_x"] = x
    rec["dc_099"] = core.discount_cumsum(x, 0.99)
    rec["dc_09405"] = core.discount_cumsum(x, 0.99 * 0.95)

    # ---- OnlineMeanStd (utils/online_mean_std.py): obs statistics over three batches
    oms = OnlineMeanStd(shape=(34,))
    batches = [rng.normal(size=(n, 34)) * rng.uniform(0.1, 3.0, 34) + rng.normal(size=34) for n in (100, 57, 1000)]
    for k, b in enumerate(batches):
        rec[f"oms_batch{k}"] = b.astype(np.float32)
        oms.update(torch.as_tensor(b, dtype=torch.float32))
        rec[f"oms_mean{k}"] = oms.mean.detach().numpy().copy()
        rec[f"oms_std{k}"] = oms.std.detach().numpy().copy()
    probe = (rng.normal(size=(16, 34)) * 5).astype(np.float32)
    rec["oms_probe"] = probe
    rec["oms_probe_out"] = oms(torch.as_tensor(probe)).numpy()
    rec["oms_probe_out_clip"] = oms(torch.as_tensor(probe), clip=True).numpy()

    # ---- ActorCritic with the PPO defaults (core.py:314-412), standardized obs + reward scaling
    params = defaults()
    obs_space = sys.modules["gym"].spaces.Box(-1000.0, 1000.0, shape=(34,), dtype=np.float32)
    act_space = sys.modules["gym"].spaces.Box(-1.0, 1.0, shape=(4,), dtype=np.float32)
    torch.manual_seed(7)
    ac = core.ActorCritic(actor_type=params["actor"], observation_space=obs_space, action_space=act_space,
                          ac_kwargs=params["ac_kwargs"], use_standardized_obs=True, use_scaled_rewards=True)
    for b in batches:
        ac.obs_oms.update(torch.as_tensor(b, dtype=torch.float32))
    rets = rng.normal(size=500) * 40.0 - 100.0
    ac.ret_oms.update(torch.as_tensor(rets, dtype=torch.float32))
    for name, t in ac.state_dict().items():
        rec["ac__" + name] = t.detach().numpy().copy()
    obs = (rng.normal(size=(64, 34)) * 2).astype(np.float32)
    rec["ac_obs"] = obs
    ac.eval()                                 # predict(): a = mu (core.py:284-290)
    a_det, v_det, _ = ac.step(torch.as_tensor(obs))
    rec["ac_mu"], rec["ac_v"] = a_det, v_det
    acts = (rng.normal(size=(64, 4)) * 0.5).astype(np.float32)
    rec["ac_acts"] = acts
    with torch.no_grad():
        pi = ac.pi.dist(ac.obs_oms(torch.as_tensor(obs)))
        rec["ac_logp"] = ac.pi.log_prob_from_dist(pi, torch.as_tensor(acts)).numpy()
    ac.pi.set_log_std(0.3)                    # annealed exploration noise (core.py:269-277)
    with torch.no_grad():
        pi = ac.pi.dist(ac.obs_oms(torch.as_tensor(obs)))
        rec["ac_logp_frac03"] = ac.pi.log_prob_from_dist(pi, torch.as_tensor(acts)).numpy()
    rec["ac_log_std_frac03"] = ac.pi.log_std.detach().numpy().copy()

    # ---- Buffer.finish_path (core.py:415-535): episodes ending terminal (last_val 0) or cut off
    # (last_val = V(s_T)), with and without reward scaling
    lens = [37, 50, 13, 64, 36]
    last_vals = [0.0, -3.25, 0.0, 1.5, -0.75]
    T = sum(lens)
    rew = (rng.normal(size=T) * 3 - 1).astype(np.float32)
    val = (rng.normal(size=T) * 5).astype(np.float32)
    rec["buf_lens"], rec["buf_last_vals"], rec["buf_rew"], rec["buf_val"] = np.array(lens), np.array(last_vals), rew, val
    rec["buf_ret_std"] = ac.ret_oms.std.detach().numpy().copy()
    for scaled in (False, True):
        buf = core.Buffer(actor_critic=ac, obs_dim=(34,), act_dim=(4,), size=T, gamma=0.99, lam=0.95,
                          adv_estimation_method="gae", use_scaled_rewards=scaled, standardize_env_obs=True,
                          standardize_advantages=True)
        t = 0
        for L, lv in zip(lens, last_vals):
            for _ in range(L):
                buf.store(np.zeros(34, np.float32), np.zeros(4, np.float32), rew[t], val[t], 0.0)
                t += 1
            buf.finish_path(last_val=lv)
        tag = "scaled" if scaled else "plain"
        rec[f"buf_adv_{tag}"] = buf.adv_buf.copy()
        rec[f"buf_vtarget_{tag}"] = buf.target_val_buf.copy()
        rec[f"buf_discret_{tag}"] = buf.discounted_ret_buf.copy()

    np.savez_compressed(os.path.join(HERE, "golden_f3.npz"), **rec)
    print("golden_f3.npz", os.path.getsize(os.path.join(HERE, "golden_f3.npz")), sorted(rec)[:8], "...")


if __name__ == "__main__":
    main()
