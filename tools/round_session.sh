#!/bin/bash
# One GPU-box session of the round: smoke, -m gpu tests, the bench line, rocprofv3 kernel stats
# and the PMC traffic of the headline (262 144 envs) and out-of-cache (1 Mi envs) workloads.
# Every GPU step runs under its own time limit; the first failure ends the session.
# usage: bash tools/round_session.sh TAG [steps...]   steps: smoke tests bench prof traffic (default: all)
set -o pipefail
TAG=${1:-r03}; shift
STEPS=${*:-"smoke tests bench prof traffic"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
has() { [[ " $STEPS " == *" $1 "* ]]; }
if has smoke; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if has tests; then
  timeout -k 10 1500 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
if has bench; then
  timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if has prof; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o step -- python3 bench.py --steps 1000 --warmup 1000 --no-cpu-baseline --streaming-ring 0 --oc-envs 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
  find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
  head -4 $OUT/kernel_stats.csv | cut -c1-200
fi
if has traffic; then
  bash tools/pmc_valu.sh ${TAG}_valu 262144 > $OUT/valu.log 2>&1 || { echo "valu pass failed"; tail -20 $OUT/valu.log; exit 1; }
  cp profiles/valu_issue.json $OUT/valu_issue.json
  for N in 262144 1048576; do
    bash tools/pmc_traffic.sh ${TAG}_traffic_$N $N > $OUT/traffic_$N.log 2>&1 || { echo "traffic $N failed"; tail -20 $OUT/traffic_$N.log; exit 1; }
    cp gpurun_out/${TAG}_traffic_$N/step_kernel_traffic.json profiles/step_kernel_traffic.json
  done
  cp profiles/step_kernel_traffic.json $OUT/step_kernel_traffic.json
  grep -h '"hbm_bytes_per_launch"\|"workload"' $OUT/step_kernel_traffic.json
fi
echo session done
