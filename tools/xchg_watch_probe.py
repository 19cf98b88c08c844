"""Per-step trace of the delta exchange's time-out look-ahead on one RCCL rank: for each env-step
the side capacity the host chose (crash budget + predicted time-outs), the step's resets, its
truncations and the overflow count, with a short TimeLimit so the look-ahead horizon spans most of
an episode.  Prints one JSON line per step in [--from, --to) and a summary.

  torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/xchg_watch_probe.py [--mode eager|run]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=120)
    ap.add_argument("--max-steps", type=int, default=41)
    ap.add_argument("--lookahead", type=int, default=33)
    ap.add_argument("--mode", default="eager", choices=("eager", "run"))
    ap.add_argument("--from", dest="lo", type=int, default=30)
    ap.add_argument("--to", dest="hi", type=int, default=60)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather, default_cap
    from cf2sim.vec_env import BatchedCrazyflieEnv
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    n = args.envs
    env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=3, device=dev,
                              max_episode_steps=args.max_steps)
    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=True, max_steps=args.max_steps, lookahead=args.lookahead)
    pipe.start(env.reset().clone())
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    ring = torch.rand(8, n, 4, device=dev, generator=g) * 2 - 1
    ptrs = [ring[r].data_ptr() for r in range(8)]
    budget = default_cap(n)
    ovf0 = 0
    for k in range(args.steps):
        if args.mode == "eager":
            buf, done = pipe.buffer(), pipe.done_buffer()
            env.step_raw(ptrs[k % 8], obs_ptr=buf.data_ptr(), done_ptr=done.data_ptr())
            pipe.publish()
        else:
            pipe.run(env, ptrs, 1)
        torch.cuda.synchronize()
        q, _, _, cap = pipe._where[k]
        resets = int(pipe.done[q].sum())
        trunc = int(env.trunc.sum())
        ovf = pipe.overflows()
        if args.lo <= k < args.hi or ovf != ovf0:
            print(json.dumps({"k": k, "cap": cap, "predicted": cap - budget, "resets": resets, "trunc": trunc,
                              "crashes": resets - trunc, "overflow": ovf - ovf0}), flush=True)
        ovf0 = ovf
    print(json.dumps({"summary": True, "overflows": pipe.overflows(), "watch": pipe.watch, "npred": pipe.npred}))
    pipe.close()
    env.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
