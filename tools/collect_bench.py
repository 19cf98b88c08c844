"""Per-launch time of the fused collect step (cf2_collect_step: env-step + actor-critic forward) at N
envs, HIP events on the env's stream over `--steps` launches after a random-action warm-up past the
start transient; the two-launch pair (cf2_step + cf2_policy_forward) is timed the same way, and the
whole loop in one launch (cf2_collect_rollout, K = --slabs steps per launch) per env-step.  Prints
one JSON line.  CF2SIM_LIB selects an A/B build."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    ap.add_argument("--slabs", type=int, default=32, help="rollout-storage slabs the outputs cycle through")
    args = ap.parse_args()
    from cf2sim.rollout import FusedActorCritic, MLPActorCritic
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = args.envs
    env = BatchedCrazyflieEnv(args.env_id, n, seed=0, want_final_obs=True)
    dev = env.device
    pol = FusedActorCritic(MLPActorCritic(obs_dim=env.obs_dim).to(dev), seed=0, precision="bf16x3")
    g = torch.Generator(device=dev).manual_seed(0)
    env.reset()
    wa = torch.rand(8, n, 4, device=dev, generator=g) * 2 - 1
    for k in range(args.warmup):
        env.step(wa[k % 8])
    S, od = args.slabs, env.obs_dim
    act = torch.rand(S + 1, n, 4, device=dev, generator=g) * 2 - 1
    obs, fin = torch.empty(S, n, od, device=dev), torch.empty(S, n, od, device=dev)
    rew = torch.empty(S, n, device=dev)
    val, lp = (torch.empty(S + 1, n, device=dev) for _ in range(2))
    dn, tr = (torch.empty(S, n, dtype=torch.uint8, device=dev) for _ in range(2))

    def fused(k):
        s = k % S
        assert env.collect_step_into(act[s], obs[s], rew[s], dn[s], tr[s], fin[s], pol, act[s + 1], val[s], lp[s])

    def pair(k):
        s = k % S
        env.step_into(act[s], obs[s], rew[s], dn[s], tr[s], final_obs_out=fin[s])
        pol.step_into(obs[s], act[s + 1], val[s], lp[s])

    def rollout(k):
        assert env.collect_rollout_into(act, obs, rew, dn, tr, fin, pol, val, lp)

    out = {"envs": n, "steps": args.steps, "env_id": args.env_id, "rollout_k": S}
    for name, fn, per in (("fused_us", fused, 1), ("two_launch_us", pair, 1), ("rollout_us_per_env_step", rollout, S),
                          ("fused_us_again", fused, 1)):
        calls = max(2, args.steps // per)
        for k in range(min(20, calls)):
            fn(k)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()                  # the env launches on torch's current stream
        for k in range(calls):
            fn(k)
        e1.record()
        torch.cuda.synchronize()
        out[name] = e0.elapsed_time(e1) * 1e3 / (calls * per)
    print(json.dumps(out))
    env.close()


if __name__ == "__main__":
    main()
