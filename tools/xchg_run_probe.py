"""Per env-step time of the delta observation exchange at one shard (default 32 768 envs, the
8-GPU node shard) on one RCCL rank: the env-step alone, the eager native exchange (one
cf2_xchg_env_step call per step), and batches (PipelinedObsGather.run, cf2_xchg_run: env-steps
back to back with the pack fused in, one all-gather + consume per batch).

  torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/xchg_run_probe.py [--envs N] [--steps K] [--unit G]
Prints one JSON line."""
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
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=600)
    ap.add_argument("--unit", type=int, default=16)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    ap.add_argument("--own-stream", action="store_true", help="run on a pool stream, not the null stream")
    ap.add_argument("--depth", type=int, default=2)
    ap.add_argument("--lookahead", type=int, default=None)
    ap.add_argument("--no-watch", action="store_true", help="no time-out look-ahead (no count copies)")
    ap.add_argument("--skip-eager", action="store_true")
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather
    from cf2sim.vec_env import BatchedCrazyflieEnv
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    n = args.envs
    if args.own_stream:
        torch.cuda.set_stream(torch.cuda.Stream())
    env = BatchedCrazyflieEnv(args.env_id, n, seed=0, device=dev)
    env.reset()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    ring = torch.rand(8, n, 4, device=dev, generator=g) * 2 - 1
    ptrs = [ring[r].data_ptr() for r in range(8)]
    res = {"envs": n, "steps": args.steps, "unit": args.unit, "depth": args.depth, "lookahead": args.lookahead,
           "watch": not args.no_watch}

    def timed(fn, steps):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        e0.record()
        fn(steps)
        e1.record()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e6 / steps, e0.elapsed_time(e1) * 1e3 / steps

    def plain(steps):
        for k in range(steps):
            env.step_raw(ptrs[k % 8])
    plain(args.warmup)
    res["env_step_us"], _ = timed(plain, args.steps)

    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=True, depth=args.depth, lookahead=args.lookahead,
                              max_steps=0 if args.no_watch else int(env.cfg.max_episode_steps), unit=args.unit)
    pipe.start(env.obs)
    res["exchange"] = pipe.exchange

    def eager(steps):
        for _ in range(steps):
            pipe.step_and_publish(env, ptrs[pipe.k % 8])
        pipe.drain()
    if not args.skip_eager:
        eager(args.warmup)
        import ctypes
        ns, calls = (ctypes.c_double * 7)(), ctypes.c_uint64()
        pipe._lib.cf2_xchg_host_times(pipe._xchg, ns, 7, ctypes.byref(calls), 1)
        res["eager_us"], res["eager_gpu_us"] = timed(eager, args.steps)
        pipe._lib.cf2_xchg_host_times(pipe._xchg, ns, 7, ctypes.byref(calls), 1)
        if calls.value:
            parts = ("c_call", "region_take", "env_step_launch", "fork", "all_gather", "consume_launch", "close_events")
            res["eager_host_us"] = {p: ns[i] / calls.value / 1e3 for i, p in enumerate(parts)}
            res["eager_host_us"]["python_and_rest"] = res["eager_us"] - res["eager_host_us"]["c_call"]

    def batched(steps):
        pipe.run(env, ptrs, steps)
        pipe.drain()
    # align to the unit, then warm up
    batched((-pipe.k) % args.unit + args.warmup)
    res["run_us"], res["run_gpu_us"] = timed(batched, args.steps)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    pipe.run(env, ptrs, args.steps)        # the host's issue time alone (the GPU catches up after)
    res["run_host_issue_us"] = (time.perf_counter() - t0) * 1e6 / args.steps
    pipe.drain()
    torch.cuda.synchronize()
    # a policy in the loop: step() per env-step (actions given one at a time), exchange per batch,
    # issued from a pool stream
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream())
    cnt = [0]

    def stepped(steps):
        with torch.cuda.stream(side):
            for _ in range(steps):
                pipe.step(env, ptrs[cnt[0] % 8])
                cnt[0] += 1
            pipe.flush()
            pipe.drain()
        torch.cuda.current_stream().wait_stream(side)
    stepped((-pipe.k) % args.unit + args.warmup)
    res["step_us"], _ = timed(stepped, args.steps)
    res["overflows"] = pipe.overflows()
    res["bytes_per_rank_per_step"] = pipe.bytes_per_rank_per_step
    # rows on request: all rows of the last step
    a = ring[pipe.k % 8]
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = torch.empty(n, env.obs_dim, device=dev)
    pipe.rows(a, a, a, out=out)
    e0.record()
    for _ in range(20):
        pipe.rows(a, a, a, out=out)
    e1.record()
    torch.cuda.synchronize()
    res["rows_us_all"] = e0.elapsed_time(e1) * 1e3 / 20
    pipe.close()
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
