"""Host time of the batched native exchange, piece by piece (one rank under torchrun, RCCL): where
the calling thread spends an env-step of PipelinedObsGather.run at one shard (default 32 768 envs).

  torchrun --nproc-per-node 1 --master-addr 127.0.0.1 tools/run_host_probe.py [--envs N] [--steps K]

Prints one JSON line of host microseconds (GPU work not awaited inside a timed loop):
  step_ctypes / step_packed_ctypes: one cf2_step / cf2_step_packed call through ctypes;
  xchg_run_call_per_step: the cf2_xchg_run C calls of run(), per env-step;
  run_python_per_step: the rest of run() (capacity look-ups, events, bookkeeping), per env-step;
  run_wall_per_step: run() + drain, wall clock, per env-step."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


class _Timed:
    """Attribute proxy of the native library that times cf2_xchg_run calls."""

    def __init__(self, lib):
        self._lib = lib
        self.t = 0.0
        self.calls = 0

    def __getattr__(self, name):
        f = getattr(self._lib, name)
        if name not in ("cf2_xchg_run", "cf2_xchg_env_step"):
            return f

        def timed(*a):
            t0 = time.perf_counter()
            r = f(*a)
            self.t += time.perf_counter() - t0
            self.calls += 1
            return r
        return timed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=32768)
    ap.add_argument("--steps", type=int, default=2000)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather, packed_words, PACK_SCRATCH_WORDS
    from cf2sim.vec_env import BatchedCrazyflieEnv
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    n, K = args.envs, args.steps
    env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=0, device=dev)
    env.reset()
    lib = env.lib
    ring = torch.rand(8, n, 4, device=dev) * 2 - 1
    ptrs = [ring[r].data_ptr() for r in range(8)]
    sp = env.stream
    rew, trunc, cost, level = env._raw_step_outputs()
    res = {"envs": n, "steps": K}

    def host(fn, reps):
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        dt = (time.perf_counter() - t0) * 1e6 / reps
        torch.cuda.synchronize()
        return dt

    res["step_ctypes"] = host(lambda: lib.cf2_step(env._ctx, ptrs[0], None, env.obs.data_ptr(), rew, env.done.data_ptr(),
                                                   trunc, cost, level, None, sp), K)
    cap = n
    words = packed_words(n, env.obs_dim // 2 - 4, cap)
    pk = torch.zeros(words, dtype=torch.int32, device=dev)
    scr = torch.zeros(2, PACK_SCRATCH_WORDS, dtype=torch.int32, device=dev)
    res["step_packed_ctypes"] = host(lambda: lib.cf2_step_packed(
        env._ctx, ptrs[0], env.obs.data_ptr(), rew, env.done.data_ptr(), trunc, cost, level, pk.data_ptr(),
        scr[0].data_ptr(), 64, sp), K)

    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=True, max_steps=int(env.cfg.max_episode_steps))
    pipe.start(env.obs)
    pipe.run(env, ptrs, 400)
    pipe.drain()
    torch.cuda.synchronize()
    proxy = _Timed(pipe._lib)
    pipe._lib = proxy
    t0 = time.perf_counter()
    pipe.run(env, ptrs, K)
    t_run = time.perf_counter() - t0
    pipe.drain()
    torch.cuda.synchronize()
    t_wall = time.perf_counter() - t0
    res["xchg_run_calls"] = proxy.calls
    res["xchg_run_call_per_step"] = proxy.t * 1e6 / K
    res["run_python_per_step"] = (t_run - proxy.t) * 1e6 / K
    res["run_wall_per_step"] = t_wall * 1e6 / K
    pipe._lib = proxy._lib
    # the eager path: one step_and_publish per env-step (a policy in the loop)
    pipe.run(env, ptrs, (-pipe.k) % pipe.unit)
    for _ in range(100):
        pipe.step_and_publish(env, ptrs[pipe.k % 8])
    pipe.drain()
    torch.cuda.synchronize()
    proxy2 = _Timed(pipe._lib)
    pipe._lib = proxy2
    t0 = time.perf_counter()
    for _ in range(K // 4):
        pipe.step_and_publish(env, ptrs[pipe.k % 8])
    t_e = time.perf_counter() - t0
    pipe.drain()
    torch.cuda.synchronize()
    res["eager_call_per_step"] = proxy2.t * 1e6 / (K // 4)
    res["eager_python_per_step"] = (t_e - proxy2.t) * 1e6 / (K // 4)
    res["eager_wall_per_step"] = (time.perf_counter() - t0) * 1e6 / (K // 4)
    pipe._lib = proxy2._lib
    import cProfile
    import io
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    pipe.run(env, ptrs, K)
    pr.disable()
    pipe.drain()
    torch.cuda.synchronize()
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("tottime").print_stats(14)
    print(buf.getvalue(), file=sys.stderr)
    pipe.close()
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
