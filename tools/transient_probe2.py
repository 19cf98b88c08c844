"""Where does the start transient of a fresh 262 144-env batch come from (DESIGN.md section 4:
the first few hundred launches run 38-40 us, then 36.3)?  Three fresh batches, each timed launch
by launch (HIP events) over its first 600 env-steps:
  fresh      created, reset, stepped at once;
  idle       created, reset, then the GPU left idle for 50 ms before stepping (time alone);
  touched    created, reset, then its state read and written back 200 times through
             cf2_get_state / cf2_set_state (the same bytes, no env-steps) before stepping.
If only `touched` starts fast, the batch's memory becomes cache-resident by being accessed
(an insertion policy of the Infinity Cache), not by elapsed time or by the env's dynamics.
Each batch is freed before the next is created."""
import gc
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def run(env, acts, steps):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    for k in range(steps):
        ev[k][0].record(s)
        env.step_raw(acts[k % 8].data_ptr())
        ev[k][1].record(s)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in ev]


def main():
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = 262144
    g = torch.Generator(device="cuda").manual_seed(1234)
    acts = torch.rand(8, n, 4, device="cuda", generator=g) * 2 - 1
    for mode in ("fresh", "idle", "touched", "fresh"):
        env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=0)
        env.reset()
        torch.cuda.synchronize()
        if mode == "idle":
            time.sleep(0.05)
        elif mode == "touched":
            for _ in range(200):
                sf, si = env.get_state()
                env.set_state(sf, si)
            torch.cuda.synchronize()
        us = run(env, acts, 600)
        segs = {f"{s}-{s + 99}": round(sum(us[s:s + 100]) / 100, 2) for s in range(0, 600, 100)}
        print(json.dumps({"mode": mode, "us_mean_per_100": segs}), flush=True)
        del env
        gc.collect()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
