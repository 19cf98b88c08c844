"""Per-wave phase timeline of one step-kernel launch (build with tools/build_variant.sh timing
-DCF2_TIMING, run with CF2SIM_LIB=build_ab/timing.so).  Prints phase durations, how waves were
placed on SIMDs, and how many waves were resident per SIMD over time.

Stamps per wave (s_memtime, shader clock, per-XCD counter): 0 entry, 1 state loads landed,
2 physics done, 3 epilogue issued, 4 block barrier, 5 resets done.  Realtime (100 MHz, global)
start/end align XCDs."""
import argparse
import ctypes
import json
import os
import sys
from collections import defaultdict

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
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
    # the small-N kernel (<= 32768 envs) runs 4 waves per 64-env block: one timing row per wave
    n_waves = (args.envs + 63) // 64 * (4 if args.envs <= 32768 else 1)
    buf = torch.zeros(n_waves, 16, dtype=torch.int64, device=env.device)
    acts = torch.rand(8, args.envs, 4, device=env.device) * 2 - 1
    for k in range(args.warmup):
        env.step_raw(acts[k % 8].data_ptr())
    torch.cuda.synchronize()
    assert lib.cf2_debug_timing_buffer(ctypes.c_void_p(buf.data_ptr())) == 0
    env.step_raw(acts[0].data_ptr())
    torch.cuda.synchronize()
    assert lib.cf2_debug_timing_buffer(ctypes.c_void_p(0)) == 0
    t = buf.cpu().numpy().astype(np.int64)
    hw = t[:, 0]
    xcc = (hw >> 32) & 0xF
    hwid = hw & 0xFFFFFFFF
    simd = (hwid >> 4) & 3
    cu = (hwid >> 8) & 0xF
    sh = (hwid >> 12) & 1
    se = (hwid >> 13) & 3
    slot = hwid & 0xF
    st = t[:, 3:12].astype(np.float64)
    # s_memtime is not synchronised across CUs: phase durations come from memtime deltas within
    # a wave, placement in time from the global 100 MHz realtime clock (x24 -> ~2.4 GHz cycles)
    res = {}
    rt0 = t[:, 1].min()
    rstart = (t[:, 1] - rt0) * 24.0
    rend = (t[:, 2] - rt0) * 24.0
    st = st - st[:, :1] + rstart[:, None]
    dur = {f"{a}->{b}": np.diff(st[:, [a, b]], axis=1)[:, 0] for a, b in [(0, 1), (1, 2), (2, 3), (3, 4), (4, 5), (0, 5)]}
    names = {"0->1": "entry->loads landed", "1->2": "physics", "2->3": "obs/history/stores",
             "3->4": "block barrier wait", "4->5": "resets+final barrier+copy", "0->5": "wave lifetime"}
    ex = t[:, 12:15].astype(np.float64)
    if (ex[:, 0] != 0).all():
        s2, s3 = t[:, 5].astype(np.float64), t[:, 6].astype(np.float64)
        print(f"  epilogue split: final sensor {np.mean(ex[:, 0] - s2):.0f}, store_core+done/reward {np.mean(ex[:, 1] - ex[:, 0]):.0f}, "
              f"history {np.mean(ex[:, 2] - ex[:, 1]):.0f}, obs stage+store_tail {np.mean(s3 - ex[:, 2]):.0f}")
    rw = t[:, 9] != 0       # waves that ran a reset (stamps 6..8)
    if rw.any():
        r6, r7, r8 = (t[rw, 9 + k].astype(np.float64) for k in range(3))
        print(f"  reset waves {int(rw.sum())}: reset_env {np.mean(r7 - r6):.0f} cycles, stores {np.mean(r8 - r7):.0f}, "
              f"barrier->reset start {np.mean(r6 - t[rw, 7]):.0f}")
    r2 = (t[:, 9] != 0) & (t[:, 11] != 0) & (t[:, 15] != 0)     # role-2 waves (stamps 6, 7, 8, 12)
    if r2.any():
        a4, r6, r7, r8, e12, e5 = (t[r2, c].astype(np.float64) for c in (7, 9, 10, 11, 15, 8))
        print(f"  role-2 waves {int(r2.sum())}: draws+barrier {np.mean(r6 - a4):.0f}, pose {np.mean(r7 - r6):.0f}, "
              f"sensor call+history {np.mean(r8 - r7):.0f}, stores+barrier {np.mean(e12 - r8):.0f}, "
              f"obs copy {np.mean(e5 - e12):.0f} cycles")
    envw = t[:, 4] != 0                     # small-N kernel: env waves stamp 1..3, helper waves 9
    if (~envw).any() and (t[~envw, 12] != 0).any():
        hw_ = ~envw & (t[:, 12] != 0)
        e = {k: t[envw, 3 + k].astype(np.float64) for k in (0, 1, 2, 3, 4, 2 + 10)}
        print(f"  small-N env waves {int(envw.sum())}: loads {np.mean(e[1] - e[0]):.0f}, physics {np.mean(e[2] - e[1]):.0f}, "
              f"obs/history/stores {np.mean(e[3] - e[2]):.0f}, -> barrier passed {np.mean(e[4] - e[3]):.0f}, "
              f"-> rows in LDS {np.mean(e[12] - e[4]):.0f}, -> end {np.mean(t[envw, 8] - t[envw, 15]):.0f}; "
              f"lifetime {np.mean(t[envw, 8] - t[envw, 3]):.0f} (p90 {np.percentile(t[envw, 8] - t[envw, 3], 90):.0f})")
        h0, h9, h4 = (t[hw_, 3 + k].astype(np.float64) for k in (0, 9, 1 + 3))
        print(f"  small-N helper waves {int(hw_.sum())}: speculative reset {np.mean(h9 - h0):.0f} "
              f"(p90 {np.percentile(h9 - h0, 90):.0f}), wait at barrier {np.mean(h4 - h9):.0f}")
        if (t[hw_, 13] != 0).all():
            h10, h11 = t[hw_, 13].astype(np.float64), t[hw_, 14].astype(np.float64)
            e_a = t[envw, 3:8].astype(np.float64)
            print(f"  small-N helpers: entry->draws in LDS {np.mean(h10 - h0):.0f} (p90 {np.percentile(h10 - h0, 90):.0f}), "
                  f"wait at draw barrier {np.mean(h11 - h10):.0f}, after it -> reset computed {np.mean(h9 - h11):.0f} "
                  f"(p90 {np.percentile(h9 - h11, 90):.0f})")
        b2 = hw_ & (t[:, 11] != 0)          # wave-2 helpers that finished a reset row (stamps 6, 8)
        if b2.any():
            c4, c6, c8, c12, c5 = (t[b2, 3 + k].astype(np.float64) for k in (4, 6, 8, 12, 2))
            print(f"  small-N wave-2 resets {int(b2.sum())}: barrier->start {np.mean(c6 - c4):.0f}, "
                  f"gyro+rows+stores {np.mean(c8 - c6):.0f} (p90 {np.percentile(c8 - c6, 90):.0f}), "
                  f"->barrier passed {np.mean(c12 - c8):.0f}, write-out {np.mean(t[b2, 8] - t[b2, 15]):.0f}")
    print(f"waves {n_waves}; span {rend.max():.0f} cycles (realtime x24); per XCD end: " +
          " ".join(f"{x}:{rend[xcc == x].max():.0f}" for x in range(8) if (xcc == x).any()))
    print("  per XCD first/last wave start: " +
          " ".join(f"{x}:{rstart[xcc == x].min():.0f}/{rstart[xcc == x].max():.0f}" for x in range(8) if (xcc == x).any()))
    for k, v in dur.items():
        print(f"  {names[k]:24s} mean {v.mean():8.0f}  p10 {np.percentile(v, 10):8.0f}  p90 {np.percentile(v, 90):8.0f}  max {v.max():8.0f}")
        res[names[k]] = float(v.mean())
    start = st[:, 0]
    # start-time histogram (rounds)
    h, edges = np.histogram(start, bins=12)
    print("  wave start histogram (cycles):", " ".join(f"{int(e)}:{c}" for e, c in zip(edges[:-1], h)))
    # residency per SIMD over time
    key = xcc * 1000 + se * 100 + sh * 50 + cu * 4 + simd
    simds = defaultdict(list)
    for w in range(n_waves):
        simds[int(key[w])].append((rstart[w], rend[w]))
    per = np.array([len(v) for v in simds.values()])
    print(f"  SIMDs used {len(simds)}; waves per SIMD min {per.min()} mean {per.mean():.2f} max {per.max()}")
    span = rend.max()
    grid = np.linspace(0, span, 200)
    occ = np.zeros_like(grid)
    for v in simds.values():
        for a, b in v:
            occ += (grid >= a) & (grid < b)
    occ /= len(simds)
    print("  mean resident waves/SIMD over time (20 buckets):",
          " ".join(f"{x:.2f}" for x in occ.reshape(20, 10).mean(1)))
    res["mean_residency"] = float(occ.mean())
    if args.out:
        json.dump(res, open(args.out, "w"), indent=1)
    env.close()


if __name__ == "__main__":
    main()
