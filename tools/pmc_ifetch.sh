#!/bin/bash
# Instruction-fetch side of the step kernels: rocprofv3 PMC passes (SQC_ICACHE_REQ / _MISSES /
# _MISSES_DUPLICATE; SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES / SQ_IFETCH / SQ_WAVES) over the bench workload
# at the node shard (32 768 envs, step_kernel_small) and at 262 144 (step_kernel); one pass per
# counter group.  usage: pmc_ifetch.sh TAG
set -o pipefail
TAG=${1:-ifetch}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 32768 262144; do
  for grp in "SQC_ICACHE_REQ SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_IFETCH SQ_WAVES"; do
    tag=$(echo $grp | cut -d' ' -f1)
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/${n}_$tag -o pmc -- python3 bench.py --steps 30 --warmup 300 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --two-streams 0 --envs-per-gpu $n > $OUT/${n}_$tag.log 2>&1 || { echo "$n $tag failed"; tail -5 $OUT/${n}_$tag.log; exit 1; }
  done
done
python3 - $OUT <<'PY'
import csv, glob, os, sys
out = sys.argv[1]
for n, kern in ((32768, "step_kernel_small"), (262144, "step_kernel<")):
    vals = {}
    for d in glob.glob(os.path.join(out, f"{n}_*")):
        if not os.path.isdir(d):
            continue
        per = {}
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                if kern in row["Kernel_Name"]:
                    key = (row["Counter_Name"], int(row["Dispatch_Id"]))
                    per[key] = per.get(key, 0.0) + float(row["Counter_Value"])
        for (c, disp), v in per.items():
            vals.setdefault(c, []).append(v)
    print(n, {c: round(sum(v[-30:]) / len(v[-30:]), 1) for c, v in sorted(vals.items())})
PY
