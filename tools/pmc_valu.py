"""VALU issue fraction from the PMC pass of tools/pmc_valu.sh.

valu_issue_frac = VALU issue cycles per SIMD / (profiled kernel duration x 2.4 GHz), where
  VALU issue cycles per SIMD = (SQ_INSTS_VALU + SQ_INSTS_VALU_TRANS_F32) * 2 / SIMDs
    (a wave64 VALU instruction occupies a SIMD-32 for 2 cycles; a transcendental twice that,
    MI355X_MICROARCH.md 'vector-instruction ISSUE cost').
1.0 would mean every SIMD issued VALU work on every cycle of the kernel at the 2.4 GHz peak
clock; under load the clock is lower, so the true fraction is somewhat higher.  The
GRBM_GUI_ACTIVE-based variant (busy cycles = GRBM_GUI_ACTIVE / 8) is kept as
valu_issue_frac_grbm: on short dispatches it implies clocks above 2.4 GHz (2.8 GHz on the 38-us
step kernel), i.e. it counts time outside the waves' lifetime, and reads low.  Step kernel: the last
30 dispatches (bench.py --steps 30 after 1000 warm-up steps); rollout kernel: every dispatch of
bench.py's fused-rollout measurement (K = 32, residency-sized slices).  Writes
profiles/valu_issue.json for bench.py."""
import csv, glob, json, os, sys

out = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024
NAMES = ["SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32", "SQ_WAVES", "GRBM_GUI_ACTIVE"]


def per_dispatch(kern, sub="pmc", names=NAMES, grid=None):
    """Counters per dispatch of kern (rows of one dispatch summed); grid: only dispatches of that
    grid size."""
    per = {}
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        for i, row in enumerate(csv.DictReader(open(f))):
            if kern in row.get("Kernel_Name", "") and row["Counter_Name"] in names:
                if grid is not None and int(row.get("Grid_Size") or row.get("Grid_Size_X") or 0) != grid:
                    continue
                key = int(row.get("Dispatch_Id") or i)
                d = per.setdefault(key, {k: 0.0 for k in names})
                d[row["Counter_Name"]] += float(row["Counter_Value"])
    return [per[k] for k in sorted(per)]


def max_grid(kern, sub="pmc"):
    """The largest grid kern was launched on in the pass: the step kernel's workload launches
    (bench.py's two_streams key launches it on half the envs)."""
    g = 0
    for f in glob.glob(os.path.join(out, sub, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kern in row.get("Kernel_Name", ""):
                g = max(g, int(row.get("Grid_Size") or row.get("Grid_Size_X") or 0))
    return g


def mfma_busy(kern, sub="pmc_mfma"):
    """MFMA-busy fraction: SQ_VALU_MFMA_BUSY_CYCLES (cycles, summed over SIMDs) / SIMDs / kernel
    cycles at 2.4 GHz, over the dispatches of the pass."""
    rows = per_dispatch(kern, sub, ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_WAVES"])
    dur = durations(kern, sub)
    if not rows or not dur:
        return None
    busy = sum(r["SQ_VALU_MFMA_BUSY_CYCLES"] for r in rows)
    return {"mfma_busy_cycles_per_simd": busy / SIMDS / len(rows),
            "mfma_busy_frac": busy / SIMDS / (sum(dur) * 1e-9 * 2.4e9)}


def durations(kern, sub="pmc", grid=None):
    """Profiled dispatch durations (ns) of kern from the kernel trace of the same pass."""
    d = []
    for f in glob.glob(os.path.join(out, sub, "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kern in row.get("Kernel_Name", "") and (grid is None or int(row.get("Grid_Size") or row.get("Grid_Size_X") or 0) == grid):
                d.append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
    return [x for _, x in sorted(d)]


def summarize(rows, label, env_steps_per_dispatch, dur_ns=None):
    s = {k: sum(r[k] for r in rows) for k in NAMES}
    issue = (s["SQ_INSTS_VALU"] + s["SQ_INSTS_VALU_TRANS_F32"]) * 2 / SIMDS
    busy = s["GRBM_GUI_ACTIVE"] / 8
    return {"kernel": label, "dispatches": len(rows),
            "valu_per_wave": s["SQ_INSTS_VALU"] / s["SQ_WAVES"],
            "trans_per_wave": s["SQ_INSTS_VALU_TRANS_F32"] / s["SQ_WAVES"],
            "valu_per_wave_per_env_step": s["SQ_INSTS_VALU"] / s["SQ_WAVES"] / env_steps_per_dispatch,
            "issue_cycles_per_simd": issue, "busy_cycles": busy, "valu_issue_frac_grbm": issue / busy,
            "valu_issue_frac": (issue / (sum(dur_ns) * 1e-9 * 2.4e9)) if dur_ns else None,
            # sanity: the clock implied by GRBM_GUI_ACTIVE over the profiled durations
            "implied_clock_GHz": (busy / (sum(dur_ns) * 1e-9) / 1e9) if dur_ns else None,
            "profiled_us_per_dispatch": (sum(dur_ns) / len(dur_ns) / 1e3) if dur_ns else None}


sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))
from cf2sim.build import _obj_key
key = _obj_key("cf2sim_kernels.hip")
# kernel names as the trace prints them (cf2::name<...>): exact, so that "rollout_kernel" does not
# also match collect_rollout_kernel
STEP, ROLL, COLL = "cf2::step_kernel<", "cf2::rollout_kernel<", "cf2::collect_kernel<"
POL = "cf2::policy_kernel<34, 1, 0>"          # the standalone policy forward (bf16x3, sampling)


def collect_entry(kern, label, steps_per_dispatch):
    rows = per_dispatch(kern, "pmc_collect")
    if not rows:
        return None
    return dict(summarize(rows, label, steps_per_dispatch, durations(kern, "pmc_collect")), **(mfma_busy(kern) or {}))


G = max_grid(STEP)
step = per_dispatch(STEP, grid=G)[-30:]
roll = per_dispatch(ROLL)
res = {"workload": f"DroneHoverBulletFreeEnvWithGust-v0:N={N}", "kernel_key": key,
       "step_kernel": summarize(step, "step_kernel", 1, durations(STEP, grid=G)[-30:]),
       "rollout_kernel": summarize(roll, "rollout_kernel (K=32)", 32, durations(ROLL)),
       "collect_kernel": collect_entry(COLL, "collect_kernel (env-step + policy)", 1),
       "policy_kernel": collect_entry(POL, "policy_kernel (actor-critic forward + sampling, 34-wide obs, bf16x3)", 1),
       "note": __doc__.split("\n\n")[1]}
prof = os.path.join(ROOT, "profiles", "valu_issue.json")
try:
    d = json.load(open(prof))
except (OSError, ValueError):
    d = {"entries": []}
d["entries"] = [e for e in d.get("entries", []) if e.get("workload") != res["workload"]] + [res]
json.dump(d, open(prof, "w"), indent=1)
json.dump(res, open(os.path.join(out, "valu_issue.json"), "w"), indent=1)
print(json.dumps({k: (v["valu_issue_frac"], v["valu_per_wave"]) for k, v in res.items() if isinstance(v, dict)}))
