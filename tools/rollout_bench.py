"""Throughput of the batched rollout caller (f3): env-steps/s of cf2sim.rollout.collect at N envs,
split into env time and policy time (HIP events)."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    ap.add_argument("--torch-policy", action="store_true", help="torch layers instead of the fused HIP policy")
    ap.add_argument("--precision", default="fp32", help="fused policy products: fp32 | bf16x3")
    ap.add_argument("--max-episode-steps", type=int, default=500, help="TimeLimit (shorter: more time-outs)")
    ap.add_argument("--no-fuse", action="store_true", help="two launches per step (cf2_step + cf2_policy_forward)")
    ap.add_argument("--env-warmup", type=int, default=1000, help="random-action env-steps before the collects")
    args = ap.parse_args()
    from cf2sim.rollout import FusedActorCritic, MLPActorCritic, collect
    from cf2sim.vec_env import BatchedCrazyflieEnv
    envs = BatchedCrazyflieEnv(args.env_id, args.envs, seed=0, want_final_obs=True,
                               max_episode_steps=args.max_episode_steps)
    ac = MLPActorCritic().cuda()
    if not args.torch_policy:
        ac = FusedActorCritic(ac, seed=0, precision=args.precision)
    g = torch.Generator(device="cuda").manual_seed(0)
    obs = envs.reset()
    wa = torch.rand(8, args.envs, 4, device="cuda", generator=g) * 2 - 1
    for k in range(args.env_warmup):     # past the synchronised-start transient
        obs = envs.step(wa[k % 8])[0]
    obs = obs.clone()
    # warm-up at the timed length: kernels, GEMM heuristics, and the caching allocator's blocks for
    # the [T, N, ...] rollout storage (a training loop collects the same T every epoch)
    ro = collect(envs, ac, args.steps, obs=obs, generator=g, fuse=not args.no_fuse)
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        ro = collect(envs, ac, args.steps, obs=ro.last_obs, generator=g, fuse=not args.no_fuse,
                     out=ro if not args.torch_policy else None)     # storage re-used, as every epoch of a training loop
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    # split: policy forward alone vs env step alone on the same sizes
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    o = ro.last_obs
    ev[0].record()
    for _ in range(args.steps):
        if args.torch_policy:
            a, v, lp = ac.step(o, generator=g)
        else:
            a, v, lp = ac.step(o)
    ev[1].record()
    for k in range(args.steps):
        envs.step(ro.act[k].contiguous())
    ev[2].record()
    torch.cuda.synchronize()
    pol_ms = ev[0].elapsed_time(ev[1]) / args.steps
    env_ms = ev[1].elapsed_time(ev[2]) / args.steps
    print(json.dumps({"rollout_env_steps_per_s": args.envs * args.steps / dt, "ms_per_step": dt / args.steps * 1e3,
                      "policy_ms_per_step": pol_ms, "env_ms_per_step": env_ms, "envs": args.envs,
                      "steps": args.steps, "env_id": args.env_id, "max_episode_steps": args.max_episode_steps,
                      "timeouts_per_step": float(ro.trunc.float().mean()) * args.envs,
                      "policy": "torch" if args.torch_policy else f"fused HIP ({args.precision})",
                      "collect_step": "two launches" if args.no_fuse or args.torch_policy else "cf2_collect_step where built"}))
    envs.close()


if __name__ == "__main__":
    main()
