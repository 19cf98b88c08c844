"""Is the start transient of a fresh 262 144-env batch (launches 0-199 of the
bench run ~39 us, the steady state 33.3 us after ~800) the GPU's clock ramping up under load, or the
batch's memory?  Fresh batches, each timed over its first 1000 env-steps (one event between
consecutive launches, per-100 means), after different preludes right before the first step:
  fresh      nothing (created, reset, stepped);
  compute    ~80 ms of compute-only work on a 16 MB operand (fp32 matmuls; the batch's memory and the
             Infinity Cache's contents are not touched beyond those 16 MB);
  other_env  1500 env-steps of a separate 32 768-env batch (the same kernel, other memory);
  sleep      80 ms of host sleep after the compute prelude (does a warmed state decay when idle?).
If `compute` and `other_env` start at the steady rate, the transient is the clock (power state),
not the batch's memory.  Each batch is freed before the next is created."""
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
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    ev[0].record(s)
    for k in range(steps):
        env.step_raw(acts[k % 8].data_ptr())
        ev[k + 1].record(s)
    torch.cuda.synchronize()
    return [ev[k].elapsed_time(ev[k + 1]) * 1e3 for k in range(steps)]


def compute_prelude(ms=80.0):
    a = torch.rand(2048, 2048, device="cuda")
    b = torch.rand(2048, 2048, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < ms:
        for _ in range(8):
            c = a @ b
        torch.cuda.synchronize()
    del a, b, c


def main():
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = 262144
    g = torch.Generator(device="cuda").manual_seed(1234)
    acts = torch.rand(8, n, 4, device="cuda", generator=g) * 2 - 1
    for mode in ("fresh", "compute", "other_env", "sleep", "fresh", "compute"):
        env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=0)
        env.reset()
        torch.cuda.synchronize()
        if mode in ("compute", "sleep"):
            compute_prelude()
            if mode == "sleep":
                time.sleep(0.08)
        elif mode == "other_env":
            o = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", 32768, seed=1)
            o.reset()
            for k in range(1500):
                o.step_raw(acts[k % 8].data_ptr())    # first 32 768 rows of the ring
            torch.cuda.synchronize()
            o.close()
        us = run(env, acts, 1000)
        segs = {f"{s}-{s + 99}": round(sum(us[s:s + 100]) / 100, 2) for s in range(0, 1000, 100)}
        first = {f"{s}-{s + 4}": round(sum(us[s:s + 5]) / 5, 2) for s in range(0, 30, 5)}
        print(json.dumps({"mode": mode, "us_mean_first_5s": first, "us_mean_per_100": segs}), flush=True)
        env.close()
        del env
        gc.collect()
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
