"""What the fused pack adds to the small-N env-step: GPU time per launch of cf2_step and of
cf2_step_packed (the same env-step with the delta exchange's pack written by the kernel), back to
back on one box, alternating blocks of launches so that drift hits both alike.

  python tools/pack_cost_probe.py [--envs N] [--reps K] [--rounds R]
Prints one JSON line of microseconds per launch (HIP events on the launch stream)."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--reps", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    ap.add_argument("--cap", type=int, default=None, help="side capacity (default: default_cap; n: no spill atomics)")
    args = ap.parse_args()
    import torch
    from cf2sim.dist import PACK_SCRATCH_WORDS, default_cap, packed_words
    from cf2sim.vec_env import BatchedCrazyflieEnv
    dev = torch.device("cuda", 0)
    n = args.envs
    env = BatchedCrazyflieEnv(args.env_id, n, seed=0, device=dev)
    env.reset()
    lib = env.lib
    ring = torch.rand(8, n, 4, device=dev) * 2 - 1
    ptrs = [ring[r].data_ptr() for r in range(8)]
    rew, trunc, cost, level = env._raw_step_outputs()
    sp = torch.cuda.current_stream(dev).cuda_stream
    ol = env.obs_dim // 2 - 4
    cap = default_cap(n) if args.cap is None else min(args.cap, n)
    pk = torch.zeros(2, packed_words(n, ol, cap), dtype=torch.int32, device=dev)
    scr = torch.zeros(2, PACK_SCRATCH_WORDS, dtype=torch.int32, device=dev)
    obs2 = torch.empty(2, n, env.obs_dim, device=dev)
    done2 = torch.empty(2, n, dtype=torch.uint8, device=dev)
    k = [0]

    def plain():
        j = k[0]
        lib.cf2_step(env._ctx, ptrs[j % 8], None, obs2[j % 2].data_ptr(), rew, done2[j % 2].data_ptr(), trunc, cost,
                     level, None, sp)
        k[0] += 1

    def packed():
        j = k[0]
        # (the counter is not re-zeroed between launches: the spill area then fills and later packs
        # drop their excess, which costs the kernel nothing extra; cf2_xchg_run zeroes it per batch)
        lib.cf2_step_packed(env._ctx, ptrs[j % 8], obs2[j % 2].data_ptr(), rew, done2[j % 2].data_ptr(), trunc, cost,
                            level, pk[j % 2].data_ptr(), scr[j % 2].data_ptr(), cap, sp)
        k[0] += 1

    host = {"plain": [], "packed": []}

    def timed(fn, name):
        import time
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            fn()
        host[name].append(round((time.perf_counter() - t0) * 1e6 / args.reps, 3))   # issue time per launch
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / args.reps

    for _ in range(300):
        plain()
    res = {"envs": n, "cap": cap, "plain_us": [], "packed_us": []}
    for _ in range(args.rounds):
        res["plain_us"].append(round(timed(plain, "plain"), 3))
        res["packed_us"].append(round(timed(packed, "packed"), 3))
    res["plain_min"], res["packed_min"] = min(res["plain_us"]), min(res["packed_us"])
    res["pack_cost_us"] = round(res["packed_min"] - res["plain_min"], 3)
    res["host_issue_us"] = host          # below the GPU time: the GPU, not the issue, sets the rate
    env.check_device_errors()
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
