"""Host time per call of the pieces of one pipelined exchange step (run under torchrun, one rank,
RCCL): what the eager per-step path of PipelinedObsGather costs on the CPU, piece by piece.
Prints one JSON line of microseconds per call (mean over --reps calls, GPU work not awaited)."""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2000)
    ap.add_argument("--envs", type=int, default=32768)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", device_id=dev)
    from cf2sim import _native
    from cf2sim.dist import PipelinedObsGather, default_cap, pack_obs, packed_words
    from cf2sim.vec_env import BatchedCrazyflieEnv
    lib = _native.load()
    n, R = args.envs, args.reps
    env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=0, device=dev)
    env.reset()
    acts = torch.rand(8, n, 4, device=dev) * 2 - 1
    cap = default_cap(n)
    words = packed_words(n, 13, cap)
    send = torch.zeros(words, dtype=torch.int32, device=dev)
    recv = torch.zeros(words, dtype=torch.int32, device=dev)
    comm = torch.cuda.Stream()
    ev = torch.cuda.Event()
    out = {}

    def t(name, fn):
        for _ in range(50):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(R):
            fn()
        out[name] = (time.perf_counter() - t0) * 1e6 / R
        torch.cuda.synchronize()

    t("step_raw", lambda: env.step_raw(acts[0].data_ptr()))
    sp = env.stream
    t("cf2_step_ctypes_only", lambda: lib.cf2_step(env._ctx, acts[0].data_ptr(), None, env.obs.data_ptr(),
                                                  env.rew.data_ptr(), env.done.data_ptr(), None, None, None, None, sp))
    t("current_stream_handle", lambda: torch.cuda.current_stream(dev).cuda_stream)
    t("tensor_index", lambda: acts[3])
    t("event_create_record", lambda: torch.cuda.Event().record(comm))
    t("event_record", lambda: ev.record(comm))
    t("stream_wait_event", lambda: comm.wait_event(ev))
    t("stream_wait_stream", lambda: comm.wait_stream(torch.cuda.current_stream()))

    def ctx():
        with torch.cuda.stream(comm):
            pass
    t("stream_context", ctx)
    scr = torch.zeros(2, 288, dtype=torch.int32, device=dev)
    t("pack_obs_checked", lambda: pack_obs(env.obs, env.done, cap, out=send, scratch=scr[0], next_scratch=scr[1]))

    def ag():
        with torch.cuda.stream(comm):
            dist.all_gather_into_tensor(recv, send, async_op=True).wait()
    t("all_gather_async_wait_in_ctx", ag)
    t("all_gather_sync", lambda: dist.all_gather_into_tensor(recv, send))
    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=True, max_steps=0)
    pipe.start(env.obs)

    def full_step():
        buf = pipe.buffer()
        env.step_raw(acts[0].data_ptr(), obs_ptr=buf.data_ptr(), done_ptr=pipe.done_buffer().data_ptr())
        pipe.publish()
    t("delta_step_eager_total", full_step)
    pipe.drain()
    if pipe.exchange == "native":         # the env-step and its exchange as one C call; a batch of 16
        ap = acts[0].data_ptr()
        t("delta_step_one_call", lambda: pipe.step_and_publish(env, ap))
        pipe.drain()
        ptrs = [acts[r].data_ptr() for r in range(8)]
        pipe.run(env, ptrs, (-pipe.k) % pipe.unit)
        t0 = time.perf_counter()
        pipe.run(env, ptrs, R - R % pipe.unit)
        out["delta_step_batched_run_host"] = (time.perf_counter() - t0) * 1e6 / (R - R % pipe.unit)
        pipe.drain()
    pipe.close()
    print(json.dumps({k: round(v, 2) for k, v in out.items()}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
