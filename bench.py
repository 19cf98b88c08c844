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

Multi-GPU: one process per GPU.  Under torchrun the ranks come from the environment; with
`--gpus N` and no launcher, bench.py starts its own N ranks as child processes before anything
touches the GPU (the role of the reference's mpi_fork, utils/mpi_tools.py:47-99).  At N > 1 the
headline is BASELINE configs[3] itself: the 262 144 envs split over the ranks (32 768 per GPU at
N = 8, contiguous global-id shards, "scaling": "strong") with the north star's RCCL all-gather of
the observations over xGMI inside the timed region -- delta rows (o_k of every env, a reset bitmap
and the reset rows' first halves; every rank advances the envs' ages and materialises any rows
bit-identically on request), 2.36x fewer xGMI bytes than the full rows, the env-steps back to back
with the pack fused into the env-step kernel and one all-gather + consume per batch of 16 on the
library's own RCCL communicator (PipelinedObsGather.run / cf2_xchg_run); `value` = 262 144 x K
env-steps / the max over ranks of the timed region.  Extra keys: "collective_free" (the same split
without the gather: the fallback headline, with "gather_obs": false and the error stated, if the
gather fails) and "weak_scaling" (every rank stepping 262 144 envs of its own).  --scaling weak
makes the weak run the headline instead (the gather then an extra key).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
XGMI_PEAK_GBS = 7 * 153.0      # 7 xGMI links x ~153 GB/s per GPU (per direction)
INFINITY_CACHE_BYTES = 256 << 20
# what one timed env-step writes: the reference's step() returns obs, reward, done and
# info{cost, disturbance_level} (envs/hover_free.py:138-166, 391-444) plus TimeLimit's truncation
BOUNDARY_OUTPUTS = ("obs", "rew", "done", "trunc", "cost", "level")
ENV_ID = "DroneHoverBulletFreeEnvWithGust-v0"
METRIC_GLOBAL_ENVS = 262144    # BASELINE.json: "262k parallel envs" for the whole node


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


def _cpu_model() -> str:
    """The host CPU's model name (name the cores the baseline ran on)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


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
    return {"value": allt, "unit": "env-steps/s", "cores": threads, "kind": "port", "cpu_model": _cpu_model(),
            "sample": f"oracle/cf2_oracle.c fp64 on {ENV_ID} (gust, noise, DR): {n_envs} envs x {steps} "
                      f"env-steps on {threads} OpenMP threads in {dtn:.1f} s; 1 thread: {one:.3g} env-steps/s "
                      f"(2048 envs x 600 env-steps, {dt1:.1f} s)"}


GATHER_TIMEOUT_S = 120      # the gather key's watchdog (bench.py measures it last at N > 1)


def step_kernel_key() -> str:
    """Content key of the step kernel's build (kernel source, headers, flags: cf2sim.build), so a
    traffic measurement stays valid across rebuilds that do not touch the step kernel."""
    from cf2sim.build import _obj_key
    return _obj_key("cf2sim_kernels.hip")


def load_traffic(workload_key: str):
    """Per-launch HBM bytes of the step kernel from rocprofv3 PMC passes (tools/pmc_traffic.sh),
    used only if they were measured on this workload with this very kernel build; otherwise None.
    profiles/step_kernel_traffic.json holds one entry per measured workload ("entries")."""
    p = os.path.join(ROOT, "profiles", "step_kernel_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        key = step_kernel_key()
        for e in d.get("entries", [d]):
            if e.get("workload") == workload_key and e.get("kernel_key") == key:
                return e.get("hbm_bytes_per_launch")
    except (OSError, ValueError, ImportError):
        pass
    return None


def load_pmc(workload_key: str) -> dict:
    """The PMC entry of tools/pmc_valu.sh (profiles/valu_issue.json) for this workload, used only if
    measured with this very kernel build; otherwise {}."""
    p = os.path.join(ROOT, "profiles", "valu_issue.json")
    try:
        with open(p) as f:
            d = json.load(f)
        key = step_kernel_key()
        for e in d.get("entries", []):
            if e.get("workload") == workload_key and e.get("kernel_key") == key:
                return e
    except (OSError, ValueError, ImportError):
        pass
    return {}


def load_valu_issue(workload_key: str, kernel: str):
    """VALU issue fraction of one kernel (step_kernel, rollout_kernel, collect_kernel,
    collect_rollout_kernel) from load_pmc, or None."""
    return (load_pmc(workload_key).get(kernel) or {}).get("valu_issue_frac")


def load_mfma_busy(workload_key: str, kernel: str):
    """MFMA-busy fraction (PMC SQ_VALU_MFMA_BUSY_CYCLES) of a fused collect kernel, or None."""
    return (load_pmc(workload_key).get(kernel) or {}).get("mfma_busy_frac")


def bytes_per_env_step(env) -> int:
    return algorithmic_bytes_per_env_step(env.cfg, outputs=BOUNDARY_OUTPUTS)


MFMA_BF16_PEAK_TFLOPS = 2500.0     # MI355X dense bf16 matrix peak (MI355X_MICROARCH.md; no sparsity)
POLICY_FLOPS_PER_ROW = 2 * (34 * 50 + 50 * 50 + 50 * 4 + 34 * 64 + 64 * 64 + 64)   # pi + V MLPs: 21 472


def secondary_roofline(hbm_bytes: float, seconds: float, valu_frac, flops: float = 0.0, mfma_busy=None) -> dict:
    """Roofline of a throughput key other than the headline step kernel: the HBM roof (algorithmic
    bytes / time against 8 TB/s), the vector-issue roof (PMC VALU issue fraction) and, with flops,
    the matrix roof (useful bf16 FLOP/s against the dense peak; mfma_busy: the PMC MFMA-busy
    fraction).  `bound` names the roof the kernel is closest to; `frac` is that fraction."""
    gbs = hbm_bytes / seconds / 1e9
    roofs = {"hbm": gbs / HBM_PEAK_GBS}
    if valu_frac is not None:
        roofs["valu"] = valu_frac
    out = {"hbm": {"achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
                   "algorithmic_bytes": hbm_bytes},
           "valu": {"issue_frac": valu_frac, "source": "PMC SQ_INSTS_VALU (+TRANS) x 2 cycles / SIMDs / kernel cycles "
                                                        "(tools/pmc_valu.sh -> profiles/valu_issue.json)"}}
    if flops:
        tf = flops / seconds / 1e12
        out["mfma"] = {"achieved": tf, "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / MFMA_BF16_PEAK_TFLOPS,
                       "useful_flops": flops, "busy_frac": mfma_busy,
                       "note": "useful FLOPs of the two MLPs; bf16x3 issues 3 bf16 MFMAs per product (and pads K)"}
        roofs["mfma"] = max(tf / MFMA_BF16_PEAK_TFLOPS, mfma_busy or 0.0)
    bound = max(roofs, key=roofs.get)
    unit = {"hbm": "GB/s", "valu": "issue fraction", "mfma": "TFLOP/s"}[bound]
    ach = {"hbm": gbs, "valu": valu_frac, "mfma": flops / seconds / 1e12 if flops else None}[bound]
    peak = {"hbm": HBM_PEAK_GBS, "valu": 1.0, "mfma": MFMA_BF16_PEAK_TFLOPS}[bound]
    out.update({"bound": bound, "achieved": ach, "peak": peak, "unit": unit, "frac": roofs[bound], "traffic": None})
    return out


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: the launcher's WORLD_SIZE, else 1); without a launcher "
                         "bench.py starts the N ranks itself")
    # BASELINE.md's protocol: 1000 warm-up env-steps, then 10 000 timed (~0.4 s of GPU time). All
    # envs start together, so the first episodes end in one synchronised auto-reset wave (around
    # env-steps 50-250); after ~1000 env-steps the reset rate is stationary (tools/reset_rate.py)
    ap.add_argument("--steps", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=1000)
    ap.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                    help="strong (default): BASELINE's --global-envs (262 144) split over the ranks, at N > 1 with the "
                         "RCCL observation all-gather in the timed region (configs[3]); weak: every rank steps 262 144 "
                         "envs of its own global ids, no data-path collective")
    ap.add_argument("--global-envs", type=int, default=METRIC_GLOBAL_ENVS,
                    help="--scaling strong: envs over the whole job, each rank stepping its contiguous shard")
    ap.add_argument("--envs-per-gpu", type=int, default=None,
                    help="weak scaling with this many envs on every rank (default 262 144)")
    ap.add_argument("--gather-obs", dest="gather_obs", action="store_true", default=None,
                    help="the north star's per-step RCCL all-gather of the observations over the 262 144 envs split "
                         "across the ranks (default: on at N > 1, where it is the headline; at N = 1 under a launcher: "
                         "one RCCL rank, the gather key)")
    ap.add_argument("--no-gather-obs", dest="gather_obs", action="store_false")
    ap.add_argument("--gather-mode", choices=("delta", "full"), default="delta",
                    help="delta: o_k + reset side slab, rows materialised on request (default); full: the rows")
    ap.add_argument("--gather-steps", type=int, default=2000,
                    help="env-steps the gather key times when the gather is not the headline (the headline times --steps)")
    ap.add_argument("--gather-envs", type=int, default=METRIC_GLOBAL_ENVS,
                    help="envs over the whole job in the gather key (split over the ranks)")
    ap.add_argument("--strong-steps", type=int, default=1000,
                    help="N > 1, --scaling weak: the strong_scaling key times 262 144 envs split over the ranks; 0 = skip")
    ap.add_argument("--weak-steps", type=int, default=1000,
                    help="N > 1, --scaling strong: the weak_scaling key times 262 144 envs on every rank; 0 = skip")
    ap.add_argument("--oc-envs", type=int, default=1 << 20,
                    help="N = 1: the out-of-cache line steps this many envs (working set far beyond the 256 MB "
                         "Infinity Cache, so state traffic is HBM traffic); 0 = skip")
    ap.add_argument("--oc-steps", type=int, default=500)
    ap.add_argument("--action-ring", type=int, default=8,
                    help="action slabs cycled through in the timed region (8 x 4 MB at 262 144 envs)")
    ap.add_argument("--two-streams", type=int, default=0,
                    help="N = 1: also time the same envs as two half contexts on two HIP streams (two_streams key; "
                         "off by default: its half-size step_kernel launches would mix into a rocprof summary "
                         "of the default run)")
    ap.add_argument("--streaming-ring", type=int, default=64,
                    help="after the timed region, 1000 env-steps with actions cycled through this many "
                         "slabs (64 x 4 MB: more than the 256 MB Infinity Cache); 0 = skip")
    ap.add_argument("--env-id", default=ENV_ID)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--graph", action="store_true", help="capture the timed steps in a hipGraph")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-envs", type=int, default=16384)
    ap.add_argument("--cpu-steps", type=int, default=1000)
    ap.add_argument("--env-kw", default="{}", help="JSON env kwargs (ablations), e.g. '{\"observation_noise\": 0}'")
    ap.add_argument("--collect-steps", type=int, default=32,
                    help="steps per collect of the f3 line (rollout.collect, fused env + policy; 0 = skip)")
    ap.add_argument("--exchange-probe", type=int, default=1,
                    help="N = 1: time the delta obs exchange's pack (one rank of the 8-GPU shape) and unpack "
                         "(all 262 144 rows) kernels on this GPU; 0 = skip")
    ap.add_argument("--rollout-k", type=int, default=32,
                    help="also time the fused K-step rollout (cf2_rollout, random actions) on 1 GPU; 0 = skip")
    return ap.parse_args(argv)


def bind_synthetic_tables(env, dev):
    """HJ-adversary envs: the reference's fastrack_{level}_15x15.npy tables are not in its checkout
    (.MISSING_LARGE_BLOBS); bind smooth synthetic 15^6 tables (one per 3 levels).  Returns the count."""
    import torch
    if int(env.cfg.disturbance) != 5:
        return 0
    nt = 3
    ax = torch.linspace(-1.0, 1.0, 15, device=dev)
    g = [ax.view([-1 if i == d else 1 for i in range(6)]) for d in range(6)]
    V = torch.stack([sum((0.3 + 0.1 * t + 0.05 * d) * g[d] ** (1 + (d + t) % 2) for d in range(6))
                     + 0.1 * torch.sin(3 * g[3] + 2 * g[4] - g[5] + t) for t in range(nt)])
    env.bind_hj_tables(V.reshape(nt, -1), [lv % nt for lv in range(int(env.cfg.num_levels))])
    return nt


def working_set_bytes(env, ring: int) -> int:
    """Bytes one env-step touches: internal state (30 float4 groups per env), the action ring and
    the boundary outputs.  Below ~256 MB they stay in the Infinity Cache between env-steps."""
    n, od = env.num_envs, env.obs_dim
    return n * 480 + ring * n * 16 + n * (4 * od + 4 + 1 + 1 + 4 + 4)


def exchange_line(args, env_kw, rank, world, dev, backend, barrier_sync, max_over_ranks, steps=None,
                  warmup=None) -> dict:
    """The north star's per-step all-gather of the observations ("RCCL all-gather over xGMI only for
    the returned observation tensor"): --gather-envs (262 144) envs split over the ranks, every
    env-step's observations made available on every rank (cf2sim.dist.PipelinedObsGather: the delta
    rows, 2.36x fewer bytes than the full rows; over RCCL the native exchange, env-steps back to back
    with the pack fused in and one all-gather + consume per batch of 16).  Timed like the headline:
    barrier + synchronize on both sides of exactly `steps` (default --gather-steps) env-steps after
    `warmup` (default --warmup), max over ranks.  The rows of the last step, materialised on every
    rank, must equal a full all-gather of them."""
    import torch
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather, delta_supported, gather_rows, shard_range
    from cf2sim.vec_env import BatchedCrazyflieEnv
    off, n = shard_range(args.gather_envs, rank, world)
    shards = [shard_range(args.gather_envs, r, world)[1] for r in range(world)]
    if len(set(shards)) != 1:
        return {"skipped": f"ragged shards {sorted(set(shards))}"}
    env = BatchedCrazyflieEnv(args.env_id, n, seed=args.seed, env_id_offset=off, device=dev, **env_kw)
    bind_synthetic_tables(env, dev)
    env.reset()
    ring = args.action_ring
    g = torch.Generator(device=dev)
    g.manual_seed(4321)
    # the job's actions, identical on every rank (a receiver builds every env's history slots from
    # them, as the policy that computed them would); a rank steps its rows [off, off + n)
    acts_g = torch.rand(ring, args.gather_envs, 4, device=dev, generator=g) * 2 - 1
    acts = acts_g[:, off:off + n]
    act_p = [acts[r].data_ptr() for r in range(ring)]
    delta = args.gather_mode == "delta" and delta_supported(env.cfg)
    # CF2SIM_RCCL_PATH: the library with RCCL's entry points the native exchange binds (default:
    # PyTorch's RCCL; the GPU tests bind their stand-in to run this path with two ranks on one GPU)
    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=delta, max_steps=int(env.cfg.max_episode_steps),
                              rccl_path=os.environ.get("CF2SIM_RCCL_PATH") or None)
    native = delta and pipe.exchange == "native"
    if delta:
        pipe.start(env.obs)

    def steps_of(steps):
        if native:
            pipe.run(env, act_p, steps)
            return
        for _ in range(steps):
            k = pipe.k
            b = pipe.buffer()
            if delta:
                env.step_raw(act_p[k % ring], obs_ptr=b.data_ptr(), done_ptr=pipe.done_buffer().data_ptr())
            else:
                env.step_raw(act_p[k % ring], obs_ptr=b.data_ptr())
            pipe.publish()

    steps = args.gather_steps if steps is None else int(steps)
    steps_of(args.warmup if warmup is None else int(warmup))
    pipe.drain()
    barrier_sync()
    t0 = time.perf_counter()
    steps_of(steps)
    pipe.drain()
    torch.cuda.synchronize()
    dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0)
    rows_check = None
    if delta:
        # rows on request: the whole [gather_envs, D] slab of the last timed step, materialised from
        # the gathered buffers and the actions, must equal a full all-gather of that step's rows
        kl = pipe.k - 1
        a3 = [acts_g[max(kl - d, 0) % ring] for d in range(3)]
        full = gather_rows(pipe.obs[pipe._where[kl][0]], sizes=shards)     # the obs buffer step kl wrote
        rows = pipe.rows(*a3)
        torch.cuda.synchronize()
        same = bool(torch.equal(rows, full))
        r0_, r1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0_.record()
        for _ in range(10):
            pipe.rows(*a3, out=rows)
        r1_.record()
        torch.cuda.synchronize()
        rows_check = {"step": kl, "rows": args.gather_envs, "equal_to_full_gather": same,
                      "us_all_rows": r0_.elapsed_time(r1_) * 1e3 / 10}
        del full, rows
    per_rank = pipe.bytes_per_rank_per_step
    rx = (world - 1) * per_rank                       # bytes this rank receives per step
    ms = el / steps * 1e3
    out = {"value": args.gather_envs * steps / el, "unit": "env-steps/s", "ms_per_step": ms,
           "steps": steps, "global_envs": args.gather_envs, "envs_per_gpu": n, "scaling": "strong",
           "mode": ("delta rows (o_k + reset bitmap + side slab of the crash budget + predicted time-outs); "
                    "every rank advances the ages, rows on request" if delta else "full rows"),
           "exchange": pipe.exchange,
           "launch": (f"env-steps back to back with the pack fused in, one all-gather + consume per batch of "
                      f"{pipe.unit} (cf2_xchg_run)" if native else "per-step publish"),
           "bytes_per_rank_per_step": per_rank, "bytes_in_per_rank_per_step": rx,
           "full_rows_bytes_per_rank_per_step": n * env.obs_dim * 4,
           "rx_GBs_per_rank": rx / (ms * 1e-3) / 1e9, "xgmi_peak_GBs": XGMI_PEAK_GBS,
           "link_bound_us_per_step": (rx / (world - 1) / (XGMI_PEAK_GBS / 7) * 1e6) if world > 1 else 0.0,
           "overflows": pipe.overflows(), "rows_on_request": rows_check}
    if rows_check is not None and not rows_check["equal_to_full_gather"]:
        out["error"] = "the exchanged rows differ from the full all-gather"     # reported, never hidden
    env.check_device_errors()
    pipe.drain()
    pipe.close()
    env.close()
    return out


def merge_gather(line: dict, info: dict, headline: bool, world: int, backend) -> dict:
    """Put the gather's result into the line.  As the headline (N > 1, BASELINE configs[3]) a
    successful gather replaces the collective-free value, step count and time per step and marks
    the config gather_obs; a failed one leaves the collective-free split as the headline
    (gather_obs false) with the error stated in config.gather_error -- never the weak figure."""
    line["gather"] = info
    if not headline:
        return line
    cf = line["config"]
    if "error" in info:
        cf["gather_obs"] = False
        cf["gather_error"] = info["error"]
        return line
    line["value"] = info["value"]
    line["ms_per_step"] = info["ms_per_step"]
    line["steps"] = info["steps"]
    cf["gather_obs"] = True
    cf.pop("gather_error", None)
    cf["workload"] += (f", the observations of every env-step all-gathered to every rank "
                       f"({info['exchange']} exchange, {info['mode'].split(' (')[0]})")
    cf["parallelism"] = (f"env-shard x{world}, {'RCCL' if backend == 'nccl' else backend} all-gather of the "
                         "observations every env-step")
    return line


def main(argv=None):
    args = parse_args(argv)
    launched = int(os.environ.get("WORLD_SIZE", "0") or 0)
    if launched == 0 and (args.gpus or 1) > 1:
        # no launcher: start the N ranks as children of this process, which never touches the GPU
        from cf2sim.dist import launch_plan, run_ranks
        plan = launch_plan(args.gpus, _free_port(), os.path.abspath(__file__), sys.argv[1:] if argv is None else argv)
        sys.exit(run_ranks(plan))
    world = launched or 1
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus}, but the launcher started {world} ranks")
    env_kw = json.loads(args.env_kw)

    import torch
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather, shard_range

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    backend = None
    # a process group at N > 1, and at N = 1 under a launcher when --gather-obs is asked for
    # explicitly (exercises the RCCL gather path on a one-GPU box)
    use_pg = world > 1 or (launched > 0 and bool(args.gather_obs))
    if use_pg:
        # one process per GPU over RCCL ("nccl"); CF2_BENCH_BACKEND=gloo rehearses the multi-rank
        # path with several ranks sharing the GPUs of a smaller box
        backend = os.environ.get("CF2_BENCH_BACKEND", "nccl")
        local_dev = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != world:
            raise SystemExit(f"bench.py: process group has {dist.get_world_size()} ranks, expected {world}")
    dev = torch.device("cuda", torch.cuda.current_device())

    from cf2sim.vec_env import BatchedCrazyflieEnv

    # the timed workload: BASELINE's metric config, 262 144 envs (C4 gust) over the whole job, each
    # rank stepping its contiguous global-id shard ("scaling": "strong"; at N = 1 all of them).  At
    # N > 1 the headline also carries the north star's per-step RCCL all-gather of the observations
    # (configs[3]); the env-steps of the shard without it are timed first here ("collective_free":
    # the headline's fallback and the step kernel's roofline at the shard size).  --scaling weak:
    # every rank steps 262 144 envs of its own, no data-path collective, the gather an extra key.
    if args.scaling == "strong" and not args.envs_per_gpu:
        off, n = shard_range(args.global_envs, rank, world)
        shards = [shard_range(args.global_envs, r, world)[1] for r in range(world)]
        scaling = "strong"
    else:
        n = args.envs_per_gpu or METRIC_GLOBAL_ENVS
        off, shards, scaling = rank * n, [n] * world, "weak"
    global_envs = sum(shards)
    gather = (world > 1) if args.gather_obs is None else bool(args.gather_obs)
    gather = gather and use_pg
    # the gather is the headline at N > 1 under strong scaling (BASELINE configs[3])
    headline_gather = gather and world > 1 and scaling == "strong"
    if headline_gather and args.gather_envs != global_envs:
        raise SystemExit("bench.py: the gathered headline splits --global-envs; pass the same --gather-envs")

    def max_over_ranks(x: float) -> float:
        if not use_pg:
            return x
        t = torch.tensor([x], device=dev if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def barrier_sync():
        if use_pg:
            dist.barrier()
        torch.cuda.synchronize()

    env = BatchedCrazyflieEnv(args.env_id, n, seed=args.seed, env_id_offset=off, device=dev, **env_kw)
    hj_tables = bind_synthetic_tables(env, dev)
    env.reset()
    ring = args.action_ring
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    acts = torch.rand(ring, n, 4, device=dev, generator=g) * 2 - 1
    stream = torch.cuda.current_stream()
    # per-step host work kept small: the action ring's addresses resolved once
    act_p = [acts[r].data_ptr() for r in range(ring)]

    def steps_of(steps):
        for k in range(steps):
            env.step_raw(act_p[k % ring])

    def run(steps, graph=None):
        """exactly `steps` env-steps between barrier + synchronize; returns the max-over-ranks wall
        time and this rank's HIP-event time on the launch stream"""
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier_sync()
        e0.record(stream)         # before the clock starts: recording costs host time, not GPU time
        t0 = time.perf_counter()
        if graph is not None:
            for g_ in graph:
                g_.replay()
        else:
            steps_of(steps)
        e1.record(stream)
        torch.cuda.synchronize()
        if use_pg:
            dist.barrier()
        return max_over_ranks(time.perf_counter() - t0), e0.elapsed_time(e1)

    steps_of(args.warmup)
    torch.cuda.synchronize()

    def capture(steps):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g_ = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g_, stream=s):
                steps_of(steps)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        return g_

    graph = [capture(args.steps)] if args.graph else None

    # ---- timed region: exactly K steps between barrier + synchronize, max over ranks ----
    elapsed, ev_ms = run(args.steps, graph)
    kern_ms = ev_ms / args.steps

    weak = None
    if world > 1 and scaling == "strong" and args.weak_steps > 0:
        # every rank stepping 262 144 envs of its own global ids, no collective (weak scaling)
        wn = METRIC_GLOBAL_ENVS
        wenv = BatchedCrazyflieEnv(args.env_id, wn, seed=args.seed, env_id_offset=rank * wn, device=dev, **env_kw)
        bind_synthetic_tables(wenv, dev)
        wenv.reset()
        wacts = torch.rand(ring, wn, 4, device=dev, generator=g) * 2 - 1
        wp = [wacts[r].data_ptr() for r in range(ring)]
        for k in range(args.warmup):
            wenv.step_raw(wp[k % ring])
        barrier_sync()
        t0 = time.perf_counter()
        for k in range(args.weak_steps):
            wenv.step_raw(wp[k % ring])
        torch.cuda.synchronize()
        dist.barrier()
        wel = max_over_ranks(time.perf_counter() - t0)
        weak = {"envs_per_gpu": wn, "global_envs": wn * world, "steps": args.weak_steps, "gather_obs": False,
                "scaling": "weak", "value": wn * world * args.weak_steps / wel, "unit": "env-steps/s",
                "ms_per_step": wel / args.weak_steps * 1e3}
        wenv.close()
        del wacts

    strong = None
    if world > 1 and scaling == "weak" and args.strong_steps > 0:
        # the same 262 144 envs split over the ranks (32 768 per GPU at N = 8), no collective
        so, sn = shard_range(METRIC_GLOBAL_ENVS, rank, world)
        senv = BatchedCrazyflieEnv(args.env_id, sn, seed=args.seed, env_id_offset=so, device=dev, **env_kw)
        bind_synthetic_tables(senv, dev)
        senv.reset()
        sacts = torch.rand(ring, sn, 4, device=dev, generator=g) * 2 - 1
        sp = [sacts[r].data_ptr() for r in range(ring)]
        for k in range(args.warmup):
            senv.step_raw(sp[k % ring])
        barrier_sync()
        t0 = time.perf_counter()
        for k in range(args.strong_steps):
            senv.step_raw(sp[k % ring])
        torch.cuda.synchronize()
        dist.barrier()
        sel = max_over_ranks(time.perf_counter() - t0)
        strong = {"envs_per_gpu": sn, "global_envs": METRIC_GLOBAL_ENVS, "steps": args.strong_steps,
                  "gather_obs": False, "value": METRIC_GLOBAL_ENVS * args.strong_steps / sel, "unit": "env-steps/s",
                  "ms_per_step": sel / args.strong_steps * 1e3}
        senv.close()
        del sacts

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
        vfr = load_valu_issue(f"{args.env_id}:N={n}", "rollout_kernel")
        # per env-step of a K-step launch: the action in and the step() outputs; the state is read
        # and written once per launch (1/K of it per env-step)
        state_b = algorithmic_bytes_per_env_step(env.cfg, outputs=()) - 16
        fb = 16 + (bytes_per_env_step(env) - state_b - 16) + state_b / K
        fused = {"value": n / (us * 1e-6), "unit": "env-steps/s", "us_per_env_step": us, "k": K,
                 "outputs": "obs, rew, done, trunc, cost, level per step (K slabs)",
                 # fraction of the kernel's cycles its SIMDs spend issuing VALU (PMC, tools/pmc_valu.sh)
                 "valu_issue_frac": vfr, "algorithmic_bytes_per_env_step": fb,
                 "roofline": secondary_roofline(fb * n, us * 1e-6, vfr)}
        del racts

    collect_line = None
    if world == 1 and args.collect_steps > 0:
        # the f3 caller: PPO/IWPG data collection (algs/iwpg/iwpg.py:372-410) over the batch with the
        # reference's default actor-critic (random init), one cf2_collect_step launch per env-step
        # (env-step + policy forward on its observations), GAE and the time-out values after the loop
        from cf2sim.rollout import FusedActorCritic, MLPActorCritic, collect
        cenv = BatchedCrazyflieEnv(args.env_id, n, seed=args.seed, device=dev, want_final_obs=True, **env_kw)
        bind_synthetic_tables(cenv, dev)
        cac = FusedActorCritic(MLPActorCritic(obs_dim=cenv.obs_dim).to(dev), seed=args.seed, precision="bf16x3")
        T = args.collect_steps
        cenv.reset()
        wact = torch.rand(8, n, 4, device=dev, generator=g) * 2 - 1
        for k in range(500):                 # past the synchronised-start transient
            cenv.step_raw(wact[k % 8].data_ptr())
        del wact
        def time_collect(mode):
            ro = collect(cenv, cac, T, obs=cenv.obs.clone(), fuse=mode)   # warm-up: kernels, storage blocks
            torch.cuda.synchronize()
            reps = 3
            t0 = time.perf_counter()
            for _ in range(reps):
                ro = collect(cenv, cac, T, obs=ro.last_obs, out=ro, fuse=mode)   # storage re-used (every epoch)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) * 1e6 / (reps * T), cenv.last_collect_fused
        # one launch per env-step first (cf2_collect_step), then the whole loop in one launch
        # (cf2_collect_rollout), the collect() default
        cus_steps, _ = time_collect("steps")
        cus, mode = time_collect(True)
        # per env-step: the env-step's bytes (action, obs, reward, done, truncation; the state once
        # per collect in the one-launch mode, every step in the per-step mode) and the policy's
        # outputs (action, value, log-probability); the policy reads the observations back from
        # L2 / LDS and its weights from LDS (staged once per launch); 21.5 kFLOP of useful MLP work
        # per row
        state_b = algorithmic_bytes_per_env_step(cenv.cfg, outputs=()) - 16
        step_b = algorithmic_bytes_per_env_step(cenv.cfg, outputs=("obs", "rew", "done", "trunc")) + 16 + 4 + 4
        one = mode is True
        cb = step_b - state_b + state_b / T if one else step_b
        wk = f"{args.env_id}:N={n}"
        # the kernel the PMC entry describes: cf2_collect_rollout runs collect_rollout_kernel_small
        # at N <= 32 768 and one collect_kernel launch per env-step above
        ck = "collect_rollout_kernel_small" if one and n <= 32768 else "collect_kernel"
        cvf = load_valu_issue(wk, ck)
        collect_line = {"value": n / (cus * 1e-6), "unit": "env-steps/s", "us_per_env_step": cus,
                        "algorithmic_bytes_per_env_step": cb, "flops_per_env_step": POLICY_FLOPS_PER_ROW,
                        "roofline": dict(secondary_roofline(cb * n, cus * 1e-6, cvf, POLICY_FLOPS_PER_ROW * n,
                                                            load_mfma_busy(wk, ck)), pmc_kernel=ck),
                        "steps_per_collect": T, "policy": "MLP actor-critic 34-50-50-4 / 34-64-64-1, bf16x3",
                        "launches": {True: "one per collect (cf2_collect_rollout)",
                                     "steps": "one per env-step (cf2_collect_step)"}.get(mode, "two per env-step"),
                        "us_per_env_step_one_launch_per_step": cus_steps,
                        # fraction of the fused kernel's SIMD cycles issuing VALU (PMC, tools/pmc_valu.sh)
                        "valu_issue_frac": cvf,
                        "includes": "env-step, policy forward + sampling, rollout storage (re-used across collects), GAE, "
                                    "time-out values"}
        cenv.close()

    two_streams = None
    if world == 1 and args.two_streams and n % 128 == 0:
        # the same envs as two contexts of n / 2 consecutive global ids, each stepping on its own HIP
        # stream with no per-step join: shard A's env-step k + 1 overlaps shard B's env-step k (the
        # launch ramp and tail of one hide under the other).  Same trajectories (split invariance).
        h = n // 2
        tstreams = [torch.cuda.Stream(device=dev) for _ in range(2)]
        halves = []
        for s_i in range(2):
            with torch.cuda.stream(tstreams[s_i]):
                he = BatchedCrazyflieEnv(args.env_id, h, seed=args.seed, device=dev, env_id_offset=s_i * h, **env_kw)
                bind_synthetic_tables(he, dev)
                he.reset()
                halves.append((he, [acts[r][s_i * h:(s_i + 1) * h].data_ptr() for r in range(ring)]))

        def two_run(k0, count):
            for k in range(k0, k0 + count):
                for s_i, (he, ptrs) in enumerate(halves):
                    with torch.cuda.stream(tstreams[s_i]):
                        he.step_raw(ptrs[k % ring])
        two_run(0, max(args.warmup, 200))
        torch.cuda.synchronize()
        t0_, t1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0_.record(stream)
        for st_ in tstreams:
            st_.wait_event(t0_)
        two_run(0, args.steps)
        for st_ in tstreams:
            ev_ = torch.cuda.Event()
            ev_.record(st_)
            stream.wait_event(ev_)
        t1_.record(stream)
        torch.cuda.synchronize()
        tus = t0_.elapsed_time(t1_) * 1e3 / args.steps
        two_streams = {"value": n / (tus * 1e-6), "unit": "env-steps/s", "us_per_env_step": tus,
                       "hbm_frac": bytes_per_env_step(env) * n / (tus * 1e-6) / 1e9 / HBM_PEAK_GBS,
                       "note": f"the same {n} envs as two contexts of {h} (consecutive global ids) on two HIP streams, "
                               "no join per env-step (the headline keeps one context on one stream)"}
        for he, _ in halves:
            he.close()
        del halves

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
                     "value": n / (sus * 1e-6), "unit": "env-steps/s", "cache_resident": False,
                     "hbm_frac": bytes_per_env_step(env) * n / (sus * 1e-6) / 1e9 / HBM_PEAK_GBS}
        del sacts

    from cf2sim.dist import delta_supported
    exchange = None
    if world == 1 and args.exchange_probe and n == METRIC_GLOBAL_ENVS and delta_supported(env.cfg):
        # the delta obs exchange of the 8-GPU shape on one GPU: 8 shards of this step's real rows
        # and done flags packed as the ranks would (cf2_obs_pack, 32 768 rows each), then a rank's
        # per-step consume of all 262 144 envs (cf2_obs_consume: the ages) and, on request, the
        # materialisation of all 262 144 rows (cf2_obs_rows), timed with HIP events on this stream
        from cf2sim.dist import PACK_SCRATCH_WORDS, consume_obs, default_cap, obs_rows, pack_obs, packed_words
        W8, n8, ol = 8, n // 8, env.obs_dim // 2 - 4
        cap = default_cap(n8)
        words = packed_words(n8, ol, cap)
        send = torch.zeros(W8 * words, dtype=torch.int32, device=dev)
        prev_pk = torch.zeros(W8 * words, dtype=torch.int32, device=dev)
        rows, dn = env.obs.clone(), env.done.clone()
        out_rows = torch.empty_like(rows)
        age = torch.full((n,), 3, dtype=torch.int16, device=dev)          # uint16 storage, as the exchange keeps it
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        reps = 20

        scr = torch.zeros(W8 + 1, PACK_SCRATCH_WORDS, dtype=torch.int32, device=dev)

        def pack_all(dst):
            for r in range(W8):
                # each pack zeroes the side-slot counters of the next one, as the ranks' packs do
                pack_obs(rows[r * n8:(r + 1) * n8], dn[r * n8:(r + 1) * n8], cap, out=dst[r * words:(r + 1) * words],
                         scratch=scr[r], next_scratch=scr[r + 1])
            scr[0].zero_()
        pack_all(prev_pk)
        torch.cuda.synchronize()
        ev[0].record(stream)
        for _ in range(reps):
            pack_all(send)
        ev[1].record(stream)
        for _ in range(reps):
            consume_obs(send, W8, n8, ol, cap, age)
        ev[2].record(stream)
        for _ in range(reps):
            obs_rows(send, cap, prev_pk, cap, W8, n8, ol, age, acts[2], acts[1], acts[0], out=out_rows)
        ev[3].record(stream)
        torch.cuda.synchronize()
        pack_us = ev[0].elapsed_time(ev[1]) * 1e3 / (reps * W8)
        consume_us = ev[1].elapsed_time(ev[2]) * 1e3 / reps
        rows_us = ev[2].elapsed_time(ev[3]) * 1e3 / reps
        full_b, delta_b = n8 * env.obs_dim * 4, words * 4
        rows_b = n * (4 * env.obs_dim + 4 * ol + 12 * 4 + 2) + W8 * delta_b
        # the exchange path packs inside the env-step (cf2_step_packed): one node-shard context, its
        # env-step with and without the fused pack, alternating blocks of launches
        shard = BatchedCrazyflieEnv(args.env_id, n8, seed=args.seed + 1, device=dev, **env_kw)
        bind_synthetic_tables(shard, dev)
        shard.reset()
        srew, strunc, scost, slevel = shard._raw_step_outputs()
        spk = torch.zeros(words, dtype=torch.int32, device=dev)
        sscr = torch.zeros(PACK_SCRATCH_WORDS, dtype=torch.int32, device=dev)
        sact = [a[:n8].contiguous() for a in acts]
        sp = stream.cuda_stream
        lib = shard.lib

        def shard_steps(packed: bool, k: int):
            for j in range(k):
                a = sact[j % len(sact)].data_ptr()
                if packed:
                    st = lib.cf2_step_packed(shard._ctx, a, shard.obs.data_ptr(), srew, shard.done.data_ptr(), strunc,
                                             scost, slevel, spk.data_ptr(), sscr.data_ptr(), cap, sp)
                else:
                    st = lib.cf2_step(shard._ctx, a, None, shard.obs.data_ptr(), srew, shard.done.data_ptr(), strunc,
                                      scost, slevel, None, sp)
                if st != 0:
                    raise RuntimeError(f"node-shard probe: status {st}")
        shard_steps(False, 200)
        best = {False: float("inf"), True: float("inf")}
        for _ in range(4):
            for packed in (False, True):
                sscr.zero_()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                shard_steps(packed, 200)
                e1.record(stream)
                e1.synchronize()
                best[packed] = min(best[packed], e0.elapsed_time(e1) * 1e3 / 200)
        shard.check_device_errors()
        shard.close()
        exchange = {"shape": f"8 ranks x {n8} envs", "cap_per_rank": cap, "bytes_per_rank_per_step": delta_b,
                    "full_rows_bytes_per_rank_per_step": full_b, "reduction": full_b / delta_b,
                    "link_bound_us_8gpu": delta_b / 153e9 * 1e6, "link_bound_us_8gpu_full_rows": full_b / 153e9 * 1e6,
                    "node_shard_step_us": best[False], "node_shard_step_packed_us": best[True],
                    "standalone_pack_us_per_rank": pack_us, "consume_us_all_envs": consume_us,
                    "consume_algorithmic_bytes": n * 4 + W8 * ((n8 + 31) // 32) * 4,
                    "rows_on_request_us_all_rows": rows_us, "rows_algorithmic_bytes": rows_b,
                    "rows_GBs": rows_b / (rows_us * 1e-6) / 1e9,
                    "note": "link bound: each GPU receives one packed buffer from each of 7 peers over its 7 xGMI links "
                            "(~153 GB/s each) in parallel; the exchange path packs inside the env-step "
                            "(node_shard_step_packed_us vs node_shard_step_us; the standalone pack kernel is the "
                            "per-step publish's); per step a receiver only advances the envs' ages (consume); "
                            "rows are materialised on request"}
        del send, prev_pk, rows, out_rows

    bytes_per = bytes_per_env_step(env)
    out_of_cache = None
    if world == 1 and args.oc_envs > 0:
        # out of the Infinity Cache: at 1 Mi envs the env state alone is ~500 MB, so every env-step
        # reads and writes it in HBM (the PMC byte counters, which include Infinity-Cache hits, then
        # measure HBM traffic: profiles/, tools/pmc_traffic.sh)
        on = args.oc_envs
        oenv = BatchedCrazyflieEnv(args.env_id, on, seed=args.seed, device=dev, **env_kw)
        bind_synthetic_tables(oenv, dev)
        oenv.reset()
        oacts = torch.rand(ring, on, 4, device=dev, generator=g) * 2 - 1
        for k in range(200):
            oenv.step_raw(oacts[k % ring].data_ptr())
        o0, o1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        o0.record(stream)
        for k in range(args.oc_steps):
            oenv.step_raw(oacts[k % ring].data_ptr())
        o1.record(stream)
        torch.cuda.synchronize()
        ous = o0.elapsed_time(o1) * 1e3 / args.oc_steps
        oach = bytes_per * on / (ous * 1e-6) / 1e9
        otraffic = load_traffic(f"{args.env_id}:N={on}")
        out_of_cache = {"envs": on, "working_set_bytes": working_set_bytes(oenv, ring), "cache_resident": False,
                        "kernel_us_per_launch": ous, "value": on / (ous * 1e-6), "unit": "env-steps/s",
                        "achieved": oach, "frac": oach / HBM_PEAK_GBS,
                        "traffic": otraffic, "traffic_ratio": (otraffic / (bytes_per * on)) if otraffic else None}
        oenv.close()
        del oacts
        # the box's own HBM rates (the peak re-measured with STREAM-style
        # kernels, cf2_hbm_probe): a read-only stream and a copy over 2 GiB buffers, far beyond the
        # 256 MB Infinity Cache.  The env-step reads ~58 % and writes ~42 % of its bytes; a plain
        # copy (50/50) runs slower than it, the read stream is the highest rate the box sustains
        from cf2sim import _native
        lib = _native.load()
        src = torch.empty(1 << 29, dtype=torch.float32, device=dev).fill_(1.0)
        dstc = torch.empty_like(src)
        sptr = torch.cuda.current_stream(dev).cuda_stream

        def probe_gbs(mode):
            for _ in range(3):
                _native.check(lib.cf2_hbm_probe(dstc.data_ptr(), src.data_ptr(), src.numel() * 4, mode, sptr), "cf2_hbm_probe")
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            c0.record(stream)
            for _ in range(10):
                _native.check(lib.cf2_hbm_probe(dstc.data_ptr(), src.data_ptr(), src.numel() * 4, mode, sptr), "cf2_hbm_probe")
            c1.record(stream)
            torch.cuda.synchronize()
            return 10 * (2 if mode == 0 else 1) * src.numel() * 4 / (c0.elapsed_time(c1) * 1e-3) / 1e9
        copy_gbs, read_gbs = probe_gbs(0), probe_gbs(1)
        del src, dstc
        out_of_cache["measured_hbm_copy_GBs"] = copy_gbs
        out_of_cache["measured_hbm_read_GBs"] = read_gbs
        out_of_cache["frac_of_measured_hbm"] = oach / max(copy_gbs, read_gbs)

    value = global_envs * args.steps / elapsed
    achieved_gbs = bytes_per * n / (kern_ms * 1e-3) / 1e9
    traffic = load_traffic(f"{args.env_id}:N={n}")
    wset = working_set_bytes(env, ring)
    line = None
    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.cpu_envs, args.cpu_steps)
        line = {
            "metric": "env-steps/sec (whole node) at 262k parallel envs; achieved HBM GB/s vs peak",
            "value": value,
            "unit": "env-steps/s",
            "n_gpus": world,
            "world_size": world,
            "backend": backend,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: uniform(-1,1) actions, Philox-seeded resets/noise/gusts"
                    + (f", {hj_tables} synthetic 15^6 HJ value tables" if hj_tables else ""),
            "config": {"workload": f"{args.env_id} ({describe(env.cfg)}), {global_envs} envs over {world} GPU(s)"
                                   f" ({n} per GPU)",
                       "envs_per_gpu": n, "global_envs": global_envs, "aggregate_phy_steps": 2,
                       "parallelism": f"env-shard x{world}, no data-path collective",
                       "gather_obs": bool(gather) and not headline_gather,
                       "graph": bool(args.graph)},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS,
                         "traffic": traffic,
                         "traffic_source": "rocprofv3 PMC FETCH_SIZE/WRITE_SIZE passes of this kernel build "
                                           "(tools/pmc_traffic.sh -> profiles/step_kernel_traffic.json)" if traffic else None,
                         "valu_issue_frac": load_valu_issue(f"{args.env_id}:N={n}", "step_kernel"),
                         "algorithmic_bytes_per_env_step": bytes_per,
                         "kernel_ms_per_launch": kern_ms,
                         "working_set_bytes": wset,
                         "cache_resident": wset < INFINITY_CACHE_BYTES,
                         "out_of_cache": out_of_cache},
            "cpu_baseline": cpu,
            "gather": None,
            "collective_free": None,
            "strong_scaling": strong,
            "weak_scaling": weak,
            "fused_rollout": fused,
            "collect": collect_line,
            "streaming_actions": streaming,
            "two_streams": two_streams,
            "delta_exchange": exchange,
        }
    if line is not None and headline_gather:
        # the collective-free split stands as the headline until the gathered run has succeeded
        line["collective_free"] = {"value": value, "unit": "env-steps/s", "steps": args.steps,
                                   "ms_per_step": elapsed / args.steps * 1e3, "kernel_ms_per_launch": kern_ms,
                                   "envs_per_gpu": n, "global_envs": global_envs, "gather_obs": False}
        line["config"]["gather_error"] = "the gathered run had not completed"
    if gather:
        # measured last, under a watchdog: the line above is complete without it, and a rank that
        # fails or stalls inside the exchange's collectives must not cost the line
        import threading

        def stalled():
            # a stalled collective: the line goes out with the collective-free headline and the
            # error stated, and the process ends non-zero so the stall is visible to the caller
            if line is not None:
                line["gather"] = {"error": f"no result after {GATHER_TIMEOUT_S} s"}
                if headline_gather:
                    line["config"]["gather_error"] = line["gather"]["error"]
                print(json.dumps(line), flush=True)
            os._exit(3)
        dog = threading.Timer(GATHER_TIMEOUT_S, stalled)
        dog.daemon = True
        dog.start()
        try:
            if headline_gather:
                # BASELINE configs[3]: exactly --steps env-steps of the split envs after --warmup,
                # the all-gather of every env-step's observations inside the timed region
                gather_info = exchange_line(args, env_kw, rank, world, dev, backend, barrier_sync, max_over_ranks,
                                            steps=args.steps, warmup=args.warmup)
            else:
                gather_info = exchange_line(args, env_kw, rank, world, dev, backend, barrier_sync, max_over_ranks)
        except Exception as e:          # every rank reports; a stall on the others ends at the watchdog
            gather_info = {"error": repr(e)[:300]}
        dog.cancel()
        if line is not None:
            merge_gather(line, gather_info, headline_gather, world, backend)
    if line is not None:
        print(json.dumps(line), flush=True)
    env.check_device_errors()
    env.close()
    if use_pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
