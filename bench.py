#!/usr/bin/env python3
"""Throughput benchmark of the batched CrazyFlie hover env-step on MI355X.

Metric (BASELINE.json): env-steps/s for the whole node at 262 144 parallel envs, plus the
achieved HBM GB/s of the step kernel against the chip's peak.

Workload (BASELINE.json configs[3], the config the metric is quoted on; it fits one GPU):
DroneHoverBulletFreeEnvWithGust -- the reference's free-hover task (envs/hover_free.py) with
its default sensor noise, 10 % domain randomisation, motor-thrust noise, 15 ms latency and
TimeLimit(500) auto-reset, plus Philox-driven torque gusts.  One step = one env-step of every
env = 2 physics sub-steps at dt = 5 ms.  Actions: uniform(-1, 1) f32 drawn once into a ring of
8 device slabs (32 MB at 262 144 envs).  The whole working set (env state ~165 MB, action ring,
outputs) then stays within the 256 MB Infinity Cache between steps; the line's
"streaming_actions" object times the same env-step with a 64-slab ring (268 MB), where the state
streams from HBM every step, as under a training loop's fresh action and rollout buffers.

Multi-GPU: one process per GPU (torchrun); envs are independent, each rank owns
--envs-per-gpu envs with its own global id range (no collective in the data path; weak
scaling).  --gather-obs adds an RCCL all-gather of the observation slab per step.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))

HBM_PEAK_GBS = 8000.0
# what one timed env-step writes: the reference's step() returns obs, reward, done and
# info{cost, disturbance_level} (envs/hover_free.py:138-166, 391-444) plus TimeLimit's truncation
BOUNDARY_OUTPUTS = ("obs", "rew", "done", "trunc", "cost", "level")   # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
ENV_ID = "DroneHoverBulletFreeEnvWithGust-v0"


def algorithmic_bytes_per_env_step(cfg, outputs=("obs", "rew", "done")) -> int:
    """Bytes one env-step must move between HBM and the chip (state read + write once, action
    in, outputs out) for this configuration; per-episode writes (reset, DR params) excluded.
    Mirrors the SoA fields the step kernel touches (DESIGN.md 'Algorithmic bytes')."""
    noise, dr = bool(cfg.observation_noise_on), bool(cfg.domain_randomization_on)
    ol = 13 if noise else 17
    B = int(cfg.buf_size)
    held = (cfg.aggregate_phy_steps % cfg.obs_rate) != 0
    gust_or_const = cfg.disturbance in (3, 4)
    level = cfg.disturbance in (3, 5) or cfg.level_mode == 1
    persist_f = 13 + 8 + 4 * B + (6 if noise else 0) + (10 if noise and held else 0) + ol + 8
    if cfg.physics == 1:
        persist_f += 3
    if cfg.use_motor_dynamics:
        persist_f += 4          # low words of the compensated motor state
    # DR parameters: dt, m, J[3], k0, k1, B[4], K[4] (A = 1 - B is not stored)
    rd_f = persist_f + (15 if dr else 0) + (3 if gust_or_const else 0) + (1 if level else 0)
    wr_f = persist_f + (3 if cfg.disturbance == 4 else 0)
    rd_i = 3 + (1 if level else 0) + (1 if cfg.disturbance == 4 else 0)
    wr_i = 3 + (1 if cfg.disturbance == 4 else 0)
    b = 4 * (rd_f + wr_f + rd_i + wr_i) + 16
    if cfg.disturbance == 1:
        b += 12
    od = 2 * (ol + 4)
    per_out = {"obs": 4 * od, "rew": 4, "done": 1, "trunc": 1, "cost": 4, "level": 4}
    return b + sum(per_out[o] for o in outputs)


def describe(cfg) -> str:
    """Human-readable workload summary of a cf2_config (bench config string)."""
    dstb = {0: "no disturbance", 1: "external disturbance", 2: "per-step uniform torque (C3)",
            3: "const wind (C2)", 4: "gust (C4)", 5: "HJ value-table disturbance"}[int(cfg.disturbance)]
    parts = [dstb]
    if cfg.num_drones > 1:
        parts.append(f"{cfg.num_drones}-drone formations{' with downwash (C5)' if cfg.downwash_on else ''}")
    parts.append("sensor noise" if cfg.observation_noise_on else "no sensor noise")
    parts.append(f"{100 * cfg.domain_randomization:.0f}% DR" if cfg.domain_randomization_on else "no DR")
    parts.append(f"{'Bullet' if cfg.physics == 0 else 'Simple'} physics x{cfg.aggregate_phy_steps} sub-steps")
    if cfg.max_episode_steps:
        parts.append(f"TimeLimit {cfg.max_episode_steps} + auto-reset")
    return ", ".join(parts)


def _host_threads() -> int:
    """Host threads this process may use (the GPU box's CPU share, not the machine's core count)."""
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and int(env) > 0:
        return int(env)
    return max(1, len(os.sched_getaffinity(0)))


def cpu_baseline(n_envs=16384, steps=1000, seed=0, threads=None):
    """Time the CPU restatement (oracle/, scalar C fp64) on a bounded sample of the same workload:
    one thread, then OpenMP over the host threads this process may use (envs split by index).
    Reported baseline only, not the target; `value` is the all-thread rate."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as orc
    from cf2sim.config import build_config
    threads = threads or _host_threads()

    def rate(n, k, t):
        env = orc.OracleEnv(build_config(ENV_ID, n, seed=seed), precision="f64")
        env.set_threads(t)
        env.reset()
        rng = np.random.default_rng(seed)
        acts = rng.uniform(-1, 1, size=(8, n, 4)).astype(np.float32)
        env.step(acts[0])                      # first touch of the outputs outside the timing
        t0 = time.perf_counter()
        for j in range(k):
            env.step(acts[j % 8])
        dt = time.perf_counter() - t0
        env.close()
        return n * k / dt, dt

    one, dt1 = rate(2048, 600, 1)
    allt, dtn = rate(n_envs, steps, threads) if threads > 1 else (one, dt1)
    return {"value": allt, "unit": "env-steps/s", "cores": threads, "kind": "port",
            "sample": f"oracle/cf2_oracle.c fp64 on {ENV_ID} (gust, noise, DR): {n_envs} envs x {steps} "
                      f"env-steps on {threads} OpenMP threads in {dtn:.1f} s; 1 thread: {one:.3g} env-steps/s "
                      f"(2048 envs x 600 env-steps, {dt1:.1f} s)"}


def step_kernel_key() -> str:
    """Content key of the step kernel's build (kernel source, headers, flags: cf2sim.build), so a
    traffic measurement stays valid across rebuilds that do not touch the step kernel."""
    from cf2sim.build import _obj_key
    return _obj_key("cf2sim_kernels.hip")


def load_traffic(workload_key: str):
    """Per-launch HBM bytes of the step kernel from rocprofv3 PMC passes (tools/pmc_traffic.sh),
    used only if they were measured on this workload with this very kernel build; otherwise None."""
    p = os.path.join(ROOT, "profiles", "step_kernel_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        if d.get("workload") == workload_key and d.get("kernel_key") == step_kernel_key():
            return d.get("hbm_bytes_per_launch")
    except (OSError, ValueError, ImportError):
        pass
    return None


def bytes_per_env_step(env) -> int:
    return algorithmic_bytes_per_env_step(env.cfg, outputs=BOUNDARY_OUTPUTS)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # BASELINE.md's protocol: 1000 warm-up env-steps, then 10 000 timed (~0.4 s of GPU time). All
    # envs start together, so the first episodes end in one synchronised auto-reset wave (around
    # env-steps 50-250); after ~1000 env-steps the reset rate is stationary (tools/reset_rate.py)
    ap.add_argument("--steps", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--envs-per-gpu", type=int, default=262144)
    ap.add_argument("--action-ring", type=int, default=8,
                    help="action slabs cycled through in the timed region (8 x 4 MB at 262 144 envs)")
    ap.add_argument("--streaming-ring", type=int, default=64,
                    help="after the timed region, 1000 env-steps with actions cycled through this many "
                         "slabs (64 x 4 MB: more than the 256 MB Infinity Cache); 0 = skip")
    ap.add_argument("--env-id", default=ENV_ID)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--gather-obs", action="store_true", help="RCCL all-gather of obs every step")
    ap.add_argument("--graph", action="store_true", help="capture the timed steps in a hipGraph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-envs", type=int, default=16384)
    ap.add_argument("--cpu-steps", type=int, default=1000)
    ap.add_argument("--env-kw", default="{}", help="JSON env kwargs (ablations), e.g. '{\"observation_noise\": 0}'")
    ap.add_argument("--rollout-k", type=int, default=32,
                    help="also time the fused K-step rollout (cf2_rollout, random actions) on 1 GPU; 0 = skip")
    args = ap.parse_args()
    env_kw = json.loads(args.env_kw)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        # one process per GPU over RCCL ("nccl"); CF2_BENCH_BACKEND=gloo rehearses the multi-rank
        # path with several ranks sharing the GPUs of a smaller box
        backend = os.environ.get("CF2_BENCH_BACKEND", "nccl")
        local_dev = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", torch.cuda.current_device())

    from cf2sim.vec_env import BatchedCrazyflieEnv

    n = args.envs_per_gpu
    env = BatchedCrazyflieEnv(args.env_id, n, seed=args.seed, env_id_offset=rank * n, device=dev, **env_kw)
    hj_tables = 0
    if int(env.cfg.disturbance) == 5:
        # HJ-adversary envs: the reference's fastrack_{level}_15x15.npy tables are not in its
        # checkout (.MISSING_LARGE_BLOBS); bind smooth synthetic 15^6 tables (one per 3 levels)
        hj_tables = 3
        ax = torch.linspace(-1.0, 1.0, 15, device=dev)
        g = [ax.view([-1 if i == d else 1 for i in range(6)]) for d in range(6)]
        V = torch.stack([sum((0.3 + 0.1 * t + 0.05 * d) * g[d] ** (1 + (d + t) % 2) for d in range(6))
                         + 0.1 * torch.sin(3 * g[3] + 2 * g[4] - g[5] + t) for t in range(hj_tables)])
        env.bind_hj_tables(V.reshape(hj_tables, -1), [lv % hj_tables for lv in range(int(env.cfg.num_levels))])
    env.reset()
    ring = args.action_ring
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    acts = torch.rand(ring, n, 4, device=dev, generator=g) * 2 - 1
    gathered = None

    def one_step(k):
        env.step_raw(acts[k % ring].data_ptr())
        if args.gather_obs and world > 1:
            dist.all_gather_into_tensor(gathered, env.obs)

    if args.gather_obs and world > 1:
        gathered = torch.empty(world * n, env.obs_dim, device=dev)
    for k in range(args.warmup):
        one_step(k)
    torch.cuda.synchronize()

    graph = None
    if args.graph:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(graph, stream=s):
                for k in range(args.steps):
                    one_step(k)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()

    # ---- timed region: exactly K steps between barrier + synchronize ----
    stream = torch.cuda.current_stream()
    ev_start, ev_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_start.record(stream)
    if graph is not None:
        graph.replay()
    else:
        for k in range(args.steps):
            one_step(k)
    ev_end.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # average step-kernel duration over the timed region, HIP events on the launch stream
    kern_ms = ev_start.elapsed_time(ev_end) / args.steps
    if world > 1:
        t = torch.tensor([elapsed], device=dev if dist.get_backend() == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if args.gather_obs and world > 1:
        # the timed region also holds the all-gathers: time the step kernel alone here
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
        for k in range(20):
            ev[k][0].record(stream)
            env.step_raw(acts[k % ring].data_ptr())
            ev[k][1].record(stream)
        torch.cuda.synchronize()
        kern_ms = sum(a.elapsed_time(b) for a, b in ev) / 20

    fused = None
    if world == 1 and args.rollout_k > 0:
        # the north star's "synthetic random-action rollouts" with the actions known in advance:
        # K env-steps per launch, the state in registers; every step's outputs written to its slab
        K = args.rollout_k
        racts = torch.rand(K, n, 4, device=dev, generator=g) * 2 - 1
        env.rollout(racts)                                   # warm-up (allocates the output slabs)
        torch.cuda.synchronize()
        reps = 3
        f0, f1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        f0.record(stream)
        for _ in range(reps):
            env.rollout(racts)
        f1.record(stream)
        torch.cuda.synchronize()
        us = f0.elapsed_time(f1) * 1e3 / (reps * K)
        fused = {"value": n / (us * 1e-6), "unit": "env-steps/s", "us_per_env_step": us, "k": K,
                 "outputs": "obs, rew, done, trunc, cost, level per step (K slabs)"}
        del racts

    streaming = None
    if world == 1 and args.streaming_ring > 0:
        # the same env-step with the actions cycled through a ring larger than the Infinity Cache
        # (as a training loop's fresh action / rollout buffers do): the env state (~165 MB at 262 144
        # envs) then no longer stays cache-resident between steps, so this is the HBM-streaming rate
        sr = args.streaming_ring
        sacts = torch.rand(sr, n, 4, device=dev, generator=g) * 2 - 1
        for k in range(2 * sr):
            env.step_raw(sacts[k % sr].data_ptr())
        s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s0.record(stream)
        for k in range(1000):
            env.step_raw(sacts[k % sr].data_ptr())
        s1.record(stream)
        torch.cuda.synchronize()
        sus = s0.elapsed_time(s1)                            # ms for 1000 launches = us per launch
        streaming = {"action_ring": sr, "action_bytes": sr * n * 16, "kernel_us_per_launch": sus,
                     "value": n / (sus * 1e-6), "unit": "env-steps/s",
                     "hbm_frac": bytes_per_env_step(env) * n / (sus * 1e-6) / 1e9 / HBM_PEAK_GBS}
        del sacts

    total_env_steps = n * args.steps * world
    value = total_env_steps / elapsed
    bytes_per = bytes_per_env_step(env)
    achieved_gbs = bytes_per * n / (kern_ms * 1e-3) / 1e9
    workload_key = f"{args.env_id}:N={n}"
    traffic = load_traffic(workload_key)

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_envs, args.cpu_steps)
        line = {
            "metric": "env-steps/sec (whole node) at 262k parallel envs; achieved HBM GB/s vs peak",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: uniform(-1,1) actions, Philox-seeded resets/noise/gusts"
                    + (f", {hj_tables} synthetic 15^6 HJ value tables" if hj_tables else ""),
            "config": {"workload": f"{args.env_id} ({describe(env.cfg)}), {n} envs per GPU",
                       "envs_per_gpu": n, "global_envs": n * world, "aggregate_phy_steps": 2,
                       "parallelism": f"env-shard x{world}", "gather_obs": bool(args.gather_obs),
                       "graph": bool(args.graph)},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "algorithmic_bytes_per_env_step": bytes_per,
                         "kernel_ms_per_launch": kern_ms},
            "cpu_baseline": cpu,
            "fused_rollout": fused,
            "streaming_actions": streaming,
        }
        print(json.dumps(line), flush=True)
    env.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
