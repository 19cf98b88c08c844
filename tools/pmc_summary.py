"""Per-dispatch means of the step kernel's PMC counters from rocprofv3 csv passes under DIR
(tools/final_round.sh writes DIR/pmc1, DIR/pmc2, ...), plus per-wave values.
usage: python tools/pmc_summary.py DIR"""
import csv
import glob
import os
import sys
from collections import defaultdict

TAIL = 30   # the timed launches (bench.py --steps 30 after its warm-up): the last 30 dispatches

per = defaultdict(dict)        # counter -> dispatch id -> value (rows of one dispatch summed)
for f in glob.glob(os.path.join(sys.argv[1], "pmc*", "**", "*counter_collection.csv"), recursive=True):
    for i, row in enumerate(csv.DictReader(open(f))):
        if "step_kernel" in row.get("Kernel_Name", ""):
            d = per[row["Counter_Name"]]
            key = int(row.get("Dispatch_Id") or i)
            d[key] = d.get(key, 0.0) + float(row["Counter_Value"])
vals = {k: [d[i] for i in sorted(d)][-TAIL:] for k, d in per.items()}
m = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(m):
    print(f"{k:32s} {m[k]:16.1f}")
w = m.get("SQ_WAVES")
if w:
    for k in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU",
              "SQ_ACTIVE_INST_VALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU"):
        if k in m:
            print(f"per-wave {k:24s} {m[k] / w:12.1f}")
