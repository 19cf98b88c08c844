"""Auto-reset rate of the bench workload over time: the fraction of envs whose episode ends at each
env-step, same env, seed and action ring as bench.py.  All envs start together, so the first
episodes end in a synchronised wave; after ~1000 env-steps the rate is stationary (BASELINE's
protocol: 1000 warm-up + 10 000 timed steps).  usage: reset_rate.py [--envs N] [--steps K]"""
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
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    args = ap.parse_args()
    from cf2sim.vec_env import BatchedCrazyflieEnv
    dev = torch.device("cuda", 0)
    n = args.envs
    env = BatchedCrazyflieEnv(args.env_id, n, seed=0, device=dev)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(1234)                      # bench.py's action ring
    acts = torch.rand(8, n, 4, device=dev, generator=g) * 2 - 1
    ends = torch.zeros(args.steps, device=dev)
    for k in range(args.steps):
        env.step_raw(acts[k % 8].data_ptr())
        ends[k] = env.done.float().sum()
    frac = (ends / n).cpu()
    windows = [(0, 50), (50, 250), (0, 1000), (1000, 2000), (1000, args.steps)]
    print(json.dumps({"env_id": args.env_id, "envs": n,
                      "episode_end_fraction_per_step": {f"{a}-{b}": round(float(frac[a:b].mean()), 5)
                                                        for a, b in windows if b <= args.steps},
                      "peak": [int(frac.argmax()), round(float(frac.max()), 4)]}))
    env.close()


if __name__ == "__main__":
    main()
