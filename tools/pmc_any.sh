#!/bin/bash
# rocprofv3 PMC pass(es) over a short bench run; prints per-dispatch means for the step kernel.
# usage: tools/pmc_any.sh TAG "CNT1 CNT2 ..." ["CNT ..." ...] -- [bench args]
set -o pipefail
TAG=$1; shift
groups=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do groups+=("$1"); shift; done
[ "$1" = "--" ] && shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for grp in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
vals = defaultdict(list)
for f in glob.glob(os.path.join(sys.argv[1], "p*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(f)):
        if "step_kernel" in row.get("Kernel_Name", ""):
            vals[row["Counter_Name"]].append(float(row["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in vals.items()}
for k in sorted(m): print(f"{k:32s} {m[k]:16.1f}")
w = m.get("SQ_WAVES")
if w:
    for k in ("SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_INSTS_VALU", "SQ_IFETCH"):
        if k in m: print(f"per-wave {k:24s} {m[k]/w:12.1f}")
PY
