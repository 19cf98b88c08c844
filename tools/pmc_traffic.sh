#!/bin/bash
# Per-launch HBM traffic of the step kernel from rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE in
# separate passes, MI355X_MICROARCH.md "HBM"), calibrated on a kernel with the same 4-byte-per-lane
# SoA access width and a known byte count (tools/membench.hip calib mode).  usage: pmc_traffic.sh TAG [ENVS]
set -o pipefail
TAG=${1:-traffic}
NENV=${2:-262144}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/calib_$c -o pmc -- ./build_ab/membench 262144 calib > $OUT/calib_$c.log 2>&1 || { echo "calib $c failed"; tail -5 $OUT/calib_$c.log; exit 1; }
  timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d $OUT/step_$c -o pmc -- python3 bench.py --steps 30 --warmup 300 --no-cpu-baseline --collect-steps 0 --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --two-streams 0 --envs-per-gpu $NENV > $OUT/step_$c.log 2>&1 || { echo "step $c failed"; tail -5 $OUT/step_$c.log; exit 1; }
done
python3 tools/pmc_traffic.py $OUT $NENV
