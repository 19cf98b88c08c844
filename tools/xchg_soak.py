"""Long-horizon check of the delta observation exchange at the node shard on one RCCL rank: many
batches of run() (synthetic actions) and then of step() (actions computed from the local rows),
across several TimeLimit periods (the synchronised time-outs at every 500th env-step included);
every `--check` env-steps the rows materialised from the exchange must equal the rows the env-step
wrote (world 1: the full gather is the rank's own rows).  Prints one JSON line.

  torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/xchg_soak.py [--envs N] [--steps K]"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=6000)
    ap.add_argument("--check", type=int, default=160)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather
    from cf2sim.vec_env import BatchedCrazyflieEnv
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    n = args.envs
    env = BatchedCrazyflieEnv(args.env_id, n, seed=11, device=dev)
    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=True, max_steps=int(env.cfg.max_episode_steps))
    pipe.start(env.reset().clone())
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    ring = torch.rand(8, n, 4, device=dev, generator=g) * 2 - 1
    ptrs = [ring[r].data_ptr() for r in range(8)]
    taken = {}
    checks, bad, resets = 0, [], 0
    t0 = time.perf_counter()
    half = args.steps // 2
    # run(): actions known ahead, batches of 16, checked every --check steps
    while pipe.k < half:
        steps = min(args.check, half - pipe.k)
        k0 = pipe.k
        for k in range(k0, k0 + steps):
            taken[k] = ring[k % 8]
        last = pipe.run(env, ptrs, steps)
        rows = pipe.rows(taken[last], taken[max(last - 1, 0)], taken[max(last - 2, 0)])
        checks += 1
        if not torch.equal(rows, pipe.local_obs()):
            bad.append(last)
        resets += int(pipe.local_done().sum())
        for old in [j for j in taken if j < pipe.k - 3]:
            del taken[old]
    # step(): a policy in the loop, actions from the local rows of the step before
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        k = pipe.k
        while k < args.steps:
            a = (torch.tanh(3.0 * pipe.local_obs()[:, 17:21]) * 0.5 + ring[k % 8] * 0.5).contiguous()
            taken[k] = a
            pipe.step(env, a.data_ptr())
            k += 1
            if k % args.check == 0 or k == args.steps:
                pipe.flush()
                last = k - 1
                rows = pipe.rows(taken[last], taken[max(last - 1, 0)], taken[max(last - 2, 0)])
                checks += 1
                if not torch.equal(rows, pipe.local_obs()):
                    bad.append(last)
            for old in [j for j in taken if j < k - 3]:
                del taken[old]
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    env.check_device_errors()
    res = {"envs": n, "steps": args.steps, "checks": checks, "mismatches": len(bad), "first_bad": bad[:3],
           "overflows": pipe.overflows(), "resets_at_checks": resets, "seconds": round(time.perf_counter() - t0, 2),
           "bytes_per_rank_per_step": pipe.bytes_per_rank_per_step,
           "time_limit": int(env.cfg.max_episode_steps)}
    pipe.close()
    env.close()
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
