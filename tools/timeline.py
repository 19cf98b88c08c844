"""Per-wave phase timeline of one env-step launch (library built with -DCF2_TIMING:
``python -c "from cf2sim.build import build_native; build_native(extra_flags=['-DCF2_TIMING'], out='build_ab/timing.so')"``,
run with ``CF2SIM_LIB=build_ab/timing.so``).  Prints phase durations, how waves were placed on
SIMDs, and how many waves were resident per SIMD over time.

Timing row per wave (16 x u64): 0 hw id (XCC << 32 | HW_ID), 1 realtime start, 2 realtime end,
3 + k = s_memtime stamp k.  Stamps (cf2sim_kernels.hip, TSTAMP):
  step_kernel (N > 32 768, one lane per env, 4 env waves per block):
    0 entry, 1 state loads landed, 2 physics done, 3 epilogue issued, 4 block barrier passed,
    6 reset role start, 7 reset pose computed, 8 role-2 sensor call + history done,
    12 every reset chunk done, 5 end
  step_kernel_small (N <= 32 768, 64 envs per block: wave 0 steps, waves 1-3 help):
    env wave:    0 entry, 1 loads landed, 2 physics done, 3 epilogue issued, 4 barrier passed,
                 12 obs rows written, 5 end
    helper wave: 0 entry, 10 step draws in LDS, 11 draw barrier passed, 9 speculative reset done,
                 4 barrier passed, 6 / 8 (wave 2, finished envs only) reset row start / done,
                 12 obs rows written, 5 end
A wave writes only the stamps of the code it runs; the others stay 0.  Every phase below is
computed over the waves that wrote both of its stamps, so a stamp a kernel never writes yields no
row (never a difference against 0).  s_memtime is per-XCD, so durations are only taken within
a wave; placement in time uses the global 100 MHz realtime clock (x24 -> ~2.4 GHz cycles)."""
import argparse
import ctypes
import json
import os
import sys
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))

LARGE_PHASES = [("loads landed", 0, 1), ("physics", 1, 2), ("obs/history/stores", 2, 3),
                ("block barrier wait", 3, 4), ("resets + obs copy", 4, 5), ("reset role: pose", 6, 7),
                ("reset role 2: sensor call + history", 7, 8), ("wave lifetime", 0, 5)]
SMALL_ENV_PHASES = [("env: loads landed", 0, 1), ("env: physics", 1, 2), ("env: obs/history/stores", 2, 3),
                    ("env: -> barrier passed", 3, 4), ("env: obs row write-out", 4, 12),
                    ("env: -> end", 12, 5), ("env: wave lifetime", 0, 5)]
SMALL_HELPER_PHASES = [("helper: entry -> step draws in LDS", 0, 10), ("helper: draw barrier wait", 10, 11),
                       ("helper: speculative reset", 11, 9), ("helper: wait at barrier", 9, 4),
                       ("helper wave 2: barrier -> reset row start", 4, 6),
                       ("helper wave 2: gyro + rows + stores", 6, 8), ("helper: reset rows + obs row write-out", 4, 12),
                       ("helper: -> end", 12, 5), ("helper: wave lifetime", 0, 5)]


def stamp(t: np.ndarray, k: int) -> np.ndarray:
    return t[:, 3 + k]


def phase(t: np.ndarray, a: int, b: int, mask=None):
    """Durations b - a over the waves (rows of t, optionally masked) that wrote both stamps;
    returns (durations, number of waves whose b preceded a, which a correct build never has)."""
    sa, sb = stamp(t, a), stamp(t, b)
    ok = (sa != 0) & (sb != 0)
    if mask is not None:
        ok &= mask
    d = (sb[ok] - sa[ok]).astype(np.float64)
    return d[d >= 0], int((d < 0).sum())


def analyze(t: np.ndarray, small: bool) -> dict:
    """Phase statistics of one launch's timing rows (pure function of the buffer; see module doc)."""
    t = np.asarray(t, dtype=np.int64)
    res = {"waves": int(t.shape[0]), "phases": {}, "negative": 0}
    if small:
        env = stamp(t, 1) != 0
        groups = [(SMALL_ENV_PHASES, env), (SMALL_HELPER_PHASES, ~env)]
    else:
        groups = [(LARGE_PHASES, None)]
    for phases, mask in groups:
        for name, a, b in phases:
            d, neg = phase(t, a, b, mask)
            res["negative"] += neg
            if d.size:
                res["phases"][name] = {"waves": int(d.size), "mean": float(d.mean()),
                                       "p10": float(np.percentile(d, 10)), "p90": float(np.percentile(d, 90)),
                                       "max": float(d.max())}
    # placement: realtime start / end of the waves that ran (realtime is global across XCDs)
    ran = (t[:, 1] != 0) & (t[:, 2] != 0)
    if ran.any():
        rt0 = t[ran, 1].min()
        rstart = (t[ran, 1] - rt0) * 24.0
        rend = (t[ran, 2] - rt0) * 24.0
        xcc = (t[ran, 0] >> 32) & 0xF
        res["span_cycles"] = float(rend.max())
        res["xcd_end"] = {int(x): float(rend[xcc == x].max()) for x in np.unique(xcc)}
        res["xcd_first_last_start"] = {int(x): [float(rstart[xcc == x].min()), float(rstart[xcc == x].max())]
                                       for x in np.unique(xcc)}
        hw = t[ran, 0] & 0xFFFFFFFF
        key = xcc * 1000 + ((hw >> 13) & 3) * 100 + ((hw >> 12) & 1) * 50 + ((hw >> 8) & 0xF) * 4 + ((hw >> 4) & 3)
        simds = defaultdict(list)
        for w in range(int(ran.sum())):
            simds[int(key[w])].append((rstart[w], rend[w]))
        per = np.array([len(v) for v in simds.values()])
        grid = np.linspace(0, max(rend.max(), 1.0), 200)
        occ = np.zeros_like(grid)
        for v in simds.values():
            for a, b in v:
                occ += (grid >= a) & (grid < b)
        occ /= len(simds)
        if small:
            # how the env waves (the ones that stamped 'loads landed') share SIMDs with each other
            env_ran = (stamp(t, 1) != 0)[ran]
            per_env = defaultdict(int)
            for w in range(int(ran.sum())):
                if env_ran[w]:
                    per_env[int(key[w])] += 1
            counts = np.bincount(np.array(list(per_env.values()), dtype=np.int64))
            res["env_waves_per_simd_hist"] = {int(c): int(n) for c, n in enumerate(counts) if n}
        res["simds_used"] = len(simds)
        res["waves_per_simd"] = [int(per.min()), float(per.mean()), int(per.max())]
        res["residency_20_buckets"] = [float(x) for x in occ.reshape(20, 10).mean(1)]
    return res


def report(res: dict) -> str:
    lines = [f"waves {res['waves']}; span {res.get('span_cycles', 0):.0f} cycles (realtime x24); "
             f"negative phase durations: {res['negative']}"]
    if "xcd_end" in res:
        lines.append("  per XCD end: " + " ".join(f"{x}:{v:.0f}" for x, v in res["xcd_end"].items()))
        lines.append("  per XCD first/last wave start: " +
                     " ".join(f"{x}:{a:.0f}/{b:.0f}" for x, (a, b) in res["xcd_first_last_start"].items()))
    for name, p in res["phases"].items():
        lines.append(f"  {name:42s} waves {p['waves']:6d}  mean {p['mean']:8.0f}  p10 {p['p10']:8.0f}  "
                     f"p90 {p['p90']:8.0f}  max {p['max']:8.0f}")
    if "simds_used" in res:
        lo, mean, hi = res["waves_per_simd"]
        lines.append(f"  SIMDs used {res['simds_used']}; waves per SIMD min {lo} mean {mean:.2f} max {hi}")
        if "env_waves_per_simd_hist" in res:
            lines.append("  SIMDs holding k env waves (k: count): " +
                         " ".join(f"{k}: {v}" for k, v in res["env_waves_per_simd_hist"].items()))
        lines.append("  mean resident waves/SIMD over time (20 buckets): " +
                     " ".join(f"{x:.2f}" for x in res["residency_20_buckets"]))
    return "\n".join(lines)


def main():
    import torch
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=262144)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env = BatchedCrazyflieEnv(args.env_id, args.envs, seed=0)
    env.reset()
    lib = env.lib
    lib.cf2_debug_timing_buffer.argtypes = [ctypes.c_void_p]
    small = args.envs <= 32768
    # the small-N kernel runs 4 waves per 64-env block: one timing row per wave
    n_waves = (args.envs + 63) // 64 * (4 if small else 1)
    buf = torch.zeros(n_waves, 16, dtype=torch.int64, device=env.device)
    acts = torch.rand(8, args.envs, 4, device=env.device) * 2 - 1
    for k in range(args.warmup):
        env.step_raw(acts[k % 8].data_ptr())
    torch.cuda.synchronize()
    assert lib.cf2_debug_timing_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    env.step_raw(acts[0].data_ptr())
    torch.cuda.synchronize()
    assert lib.cf2_debug_timing_buffer(ctypes.c_void_p(0)) == 0
    res = analyze(buf.cpu().numpy(), small)
    print(report(res))
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)
    env.close()


if __name__ == "__main__":
    main()
