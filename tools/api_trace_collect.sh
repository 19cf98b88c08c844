#!/bin/bash
# HIP API trace of the collect loop (rocprofv3 --hip-runtime-trace, no counters): which runtime
# calls run between the timed collects.  usage: api_trace_collect.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-apitrace}; mkdir -p $OUT
timeout -k 10 200 rocprofv3 --hip-runtime-trace --kernel-trace --output-format csv -d $OUT/prof -o r -- python3 tools/rollout_bench.py --precision bf16x3 --env-warmup 300 > $OUT/rb.json 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
f=$(find $OUT/prof -name "*hip_api_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
c = collections.Counter(); t = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    c[r["Function"]] += 1; t[r["Function"]] += d
for k, v in sorted(t.items(), key=lambda kv: -kv[1])[:25]:
    print(f"{k:40s} n={c[k]:6d} total {v/1e3:10.1f} us  mean {v/c[k]/1e3:8.2f} us")
PY
