#!/bin/bash
# Round-3 measurement, part A (one box session): smoke, -m gpu tests, PMC traffic of the step kernel at
# 262 144 and 1 Mi envs, VALU issue fractions (step, fused rollout, fused collect).  The JSON results
# land in gpurun_out/$TAG/ for profiles/.  usage: bash tools/r03_measure_a.sh TAG
set -o pipefail
TAG=${1:-r03a}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
bash tools/pmc_traffic.sh ${TAG}_t256k 262144 > $OUT/traffic256k.log 2>&1 || { echo "traffic failed"; tail -20 $OUT/traffic256k.log; exit 1; }
cp gpurun_out/${TAG}_t256k/step_kernel_traffic.json profiles/step_kernel_traffic.json
bash tools/pmc_traffic.sh ${TAG}_t1m 1048576 > $OUT/traffic1m.log 2>&1 || { echo "traffic 1m failed"; tail -20 $OUT/traffic1m.log; exit 1; }
cp gpurun_out/${TAG}_t1m/step_kernel_traffic.json profiles/step_kernel_traffic.json
cp profiles/step_kernel_traffic.json $OUT/step_kernel_traffic.json
bash tools/pmc_valu.sh ${TAG}_valu 262144 > $OUT/valu.log 2>&1 || { echo "valu failed"; tail -20 $OUT/valu.log; exit 1; }
cp profiles/valu_issue.json $OUT/valu_issue.json
cat $OUT/valu.log | tail -2
echo done
