"""Time the fused actor-critic forward (cf2_policy_forward) alone on random observations:
python tools/policy_bench.py [--rows N] [--iters K]"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=262144)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--obs-dim", type=int, default=34)
    ap.add_argument("--precision", default="bf16x3")
    args = ap.parse_args()
    from cf2sim.rollout import FusedActorCritic, MLPActorCritic
    ac = MLPActorCritic(obs_dim=args.obs_dim).cuda()
    fused = FusedActorCritic(ac, seed=0, precision=args.precision)
    obs = torch.randn(args.rows, args.obs_dim, device="cuda")
    act = torch.empty(args.rows, 4, device="cuda")
    val = torch.empty(args.rows, device="cuda")
    logp = torch.empty(args.rows, device="cuda")
    for _ in range(5):
        fused.step_into(obs, act, val, logp)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        fused.step_into(obs, act, val, logp)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / args.iters * 1e3
    flops = 2 * (args.obs_dim * 114 + 50 * 50 + 64 * 64 + 50 * 4 + 64) * args.rows
    print(json.dumps({"rows": args.rows, "us_per_forward": us, "useful_tflops": flops / us * 1e-6, "precision": args.precision}))


if __name__ == "__main__":
    main()
