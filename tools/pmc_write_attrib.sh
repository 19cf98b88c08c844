#!/bin/bash
# Where the step kernel's write traffic beyond its algorithmic bytes comes from: rocprofv3 PMC
# WRITE_SIZE (and FETCH_SIZE) of the bench workload at 262 144 envs with auto-reset on (the bench) and
# off (no per-episode reset writes), one pass per counter and config.  WRITE_SIZE needs no
# calibration on gfx950 (factor 1.000, tools/pmc_traffic.sh); FETCH_SIZE counts half (factor 2).
# usage: pmc_write_attrib.sh TAG
set -o pipefail
TAG=${1:-wattrib}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in reset:{} noreset:{\"auto_reset\":false}; do
  name=${cfg%%:*}; kw=${cfg#*:}
  for c in WRITE_SIZE FETCH_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/${name}_$c -o pmc -- python3 bench.py --steps 30 --warmup 300 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --two-streams 0 --envs-per-gpu 262144 --env-kw "$kw" > $OUT/${name}_$c.log 2>&1 || { echo "$name $c failed"; tail -5 $OUT/${name}_$c.log; exit 1; }
  done
done
python3 - $OUT <<'PY'
import sys, os
sys.argv = [sys.argv[0], sys.argv[1]]
sys.path.insert(0, "tools")
out = sys.argv[1]
import importlib.util
spec = importlib.util.spec_from_file_location("pt", "tools/pmc_traffic.py")
src = open("tools/pmc_traffic.py").read().split("\nN = 262144")[0]
ns = {}
exec(compile(src, "pmc_traffic_head", "exec"), ns)
for name in ("reset", "noreset"):
    w = ns["mean_counter"](os.path.join(out, f"{name}_WRITE_SIZE"), "WRITE_SIZE", "step_kernel") * 1024
    f = ns["mean_counter"](os.path.join(out, f"{name}_FETCH_SIZE"), "FETCH_SIZE", "step_kernel") * 1024 * 2
    print(f"{name}: write {w/1e6:.2f} MB ({w/262144:.1f} B/env)  read {f/1e6:.2f} MB ({f/262144:.1f} B/env)")
PY
