#!/bin/bash
# VALU issue fraction of the step kernel and the fused rollout kernel: one
# rocprofv3 PMC pass (SQ_INSTS_VALU, SQ_INSTS_VALU_TRANS_F32, SQ_WAVES, GRBM_GUI_ACTIVE) over the
# bench workload; tools/pmc_valu.py turns it into profiles/valu_issue.json.  usage: pmc_valu.sh TAG [ENVS]
set -o pipefail
TAG=${1:-valu}
NENV=${2:-262144}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o pmc -- python3 bench.py --steps 30 --warmup 1000 --no-cpu-baseline --collect-steps 0 --rollout-k 32 --streaming-ring 0 --oc-envs 0 --global-envs $NENV > $OUT/bench.log 2>&1 || { echo "pmc pass failed"; tail -5 $OUT/bench.log; exit 1; }
# the fused collect step (cf2_collect_step) on the same workload, from its own per-launch benchmark
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_collect -o pmc -- python3 tools/collect_bench.py --envs $NENV --steps 30 --warmup 600 > $OUT/collect.log 2>&1 || { echo "collect pmc pass failed"; tail -5 $OUT/collect.log; exit 1; }
python3 tools/pmc_valu.py $OUT $NENV
