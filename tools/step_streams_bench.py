"""The bench workload's env-step at N envs split into S contexts (consecutive global env ids) whose
launches go to S HIP streams: step k of shard s depends only on step k - 1 of shard s, so one
shard's launch ramp and tail overlap another shard's steady part.  Per env-step time of all N
envs (HIP events around --steps steps of every shard, after --warmup random-action steps).
Results do not depend on the split (physics keyed by the global env id).  One JSON line per S."""
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
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    args = ap.parse_args()
    from cf2sim.vec_env import BatchedCrazyflieEnv
    N = args.envs
    ring = 8
    for S in [int(x) for x in args.splits.split(",")]:
        n = N // S
        streams = [torch.cuda.Stream() for _ in range(S)]
        shards = []
        for s in range(S):
            with torch.cuda.stream(streams[s]):
                e = BatchedCrazyflieEnv(args.env_id, n, seed=0, env_id_offset=s * n)
                e.reset()
                acts = torch.rand(ring, n, 4, device="cuda") * 2 - 1
                shards.append((e, acts))
        torch.cuda.synchronize()

        def run(k0, count):
            for k in range(k0, k0 + count):
                for s, (e, acts) in enumerate(shards):
                    with torch.cuda.stream(streams[s]):
                        e.step_raw(acts[k % ring].data_ptr())

        run(0, args.warmup)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.current_stream())
        for st in streams:
            st.wait_event(e0)
        run(args.warmup, args.steps)
        for st in streams:
            ev = torch.cuda.Event()
            ev.record(st)
            torch.cuda.current_stream().wait_event(ev)
        e1.record(torch.cuda.current_stream())
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / args.steps
        print(json.dumps({"envs": N, "splits": S, "us_per_env_step": us, "env_steps_per_s": N / (us * 1e-6),
                          "steps": args.steps}), flush=True)
        for e, _ in shards:
            e.close()
        del shards


if __name__ == "__main__":
    main()
