"""Is the slow stretch after a synchronised start (launches ~50-300) a
property of the env batch or of the GPU's clocks?  Env A runs 2000 env-steps first (the GPU is
warm), then a fresh env B (same config, new seed) starts and its first 600 launches are timed one
by one with HIP events, next to the fraction of B's envs that reset at each step."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def run(env, acts, steps):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    ends = torch.zeros(steps, device="cuda")
    for k in range(steps):
        ev[k][0].record(s)
        env.step_raw(acts[k % 8].data_ptr())
        ev[k][1].record(s)
        ends[k] = env.done.float().mean()
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 for a, b in ev], ends.cpu().tolist()


def main():
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = 262144
    g = torch.Generator(device="cuda").manual_seed(1234)
    acts = torch.rand(8, n, 4, device="cuda", generator=g) * 2 - 1
    a = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=0)
    a.reset()
    run(a, acts, 2000)
    b = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=7)
    b.reset()
    us, ends = run(b, acts, 600)
    for s in range(0, 600, 50):
        seg, e = us[s:s + 50], ends[s:s + 50]
        print(json.dumps({"launches": f"{s}-{s + 49}", "us_mean": round(sum(seg) / len(seg), 2),
                          "us_min": round(min(seg), 2), "reset_frac": round(sum(e) / len(e), 4)}))
    us_a, _ = run(a, acts, 200)
    print(json.dumps({"env A after B": round(sum(us_a) / len(us_a), 2)}))


if __name__ == "__main__":
    main()
