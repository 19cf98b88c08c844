"""VALU issue fraction from the PMC pass of tools/pmc_valu.sh.

valu_issue_frac = VALU issue cycles per SIMD / kernel busy cycles, where
  VALU issue cycles per SIMD = (SQ_INSTS_VALU + SQ_INSTS_VALU_TRANS_F32) * 2 / SIMDs
    (a wave64 VALU instruction occupies a SIMD-32 for 2 cycles; a transcendental twice that,
    MI355X_MICROARCH.md 'vector-instruction ISSUE cost')
  kernel busy cycles = GRBM_GUI_ACTIVE / 8 (the counter sums the 8 XCDs).
1.0 would mean every SIMD issued VALU work on every cycle of the kernel.  Step kernel: the last
30 dispatches (bench.py --steps 30 after 1000 warm-up steps); rollout kernel: every dispatch of
bench.py's fused-rollout measurement (K = 32, residency-sized slices).  Writes
profiles/valu_issue.json for bench.py."""
import csv, glob, json, os, sys

out = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 262144
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS = 1024
NAMES = ["SQ_INSTS_VALU", "SQ_INSTS_VALU_TRANS_F32", "SQ_WAVES", "GRBM_GUI_ACTIVE"]


def per_dispatch(kern):
    per = {}
    for f in glob.glob(os.path.join(out, "pmc", "**", "*counter_collection.csv"), recursive=True):
        for i, row in enumerate(csv.DictReader(open(f))):
            if kern in row.get("Kernel_Name", "") and row["Counter_Name"] in NAMES:
                key = int(row.get("Dispatch_Id") or i)
                d = per.setdefault(key, {k: 0.0 for k in NAMES})
                d[row["Counter_Name"]] += float(row["Counter_Value"])
    return [per[k] for k in sorted(per)]


def summarize(rows, label, env_steps_per_dispatch):
    s = {k: sum(r[k] for r in rows) for k in NAMES}
    issue = (s["SQ_INSTS_VALU"] + s["SQ_INSTS_VALU_TRANS_F32"]) * 2 / SIMDS
    busy = s["GRBM_GUI_ACTIVE"] / 8
    return {"kernel": label, "dispatches": len(rows),
            "valu_per_wave": s["SQ_INSTS_VALU"] / s["SQ_WAVES"],
            "trans_per_wave": s["SQ_INSTS_VALU_TRANS_F32"] / s["SQ_WAVES"],
            "valu_per_wave_per_env_step": s["SQ_INSTS_VALU"] / s["SQ_WAVES"] / env_steps_per_dispatch,
            "issue_cycles_per_simd": issue, "busy_cycles": busy, "valu_issue_frac": issue / busy}


sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))
from cf2sim.build import _obj_key
key = _obj_key("cf2sim_kernels.hip")
step = per_dispatch("step_kernel")[-30:]
roll = per_dispatch("rollout_kernel")
res = {"workload": f"DroneHoverBulletFreeEnvWithGust-v0:N={N}", "kernel_key": key,
       "step_kernel": summarize(step, "step_kernel", 1),
       "rollout_kernel": summarize(roll, "rollout_kernel (K=32)", 32),
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
