#!/bin/bash
# VALU issue fraction of the step kernel, the fused rollout kernel and the fused collect kernel, and
# the collect kernel's MFMA-busy fraction: rocprofv3 PMC passes (SQ_INSTS_VALU, SQ_INSTS_VALU_TRANS_F32,
# SQ_WAVES, GRBM_GUI_ACTIVE; SQ_VALU_MFMA_BUSY_CYCLES) over the bench workload; tools/pmc_valu.py
# turns them into profiles/valu_issue.json.  usage: pmc_valu.sh TAG [ENVS]
set -o pipefail
TAG=${1:-valu}
NENV=${2:-262144}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o pmc -- python3 bench.py --steps 30 --warmup 300 --no-cpu-baseline --collect-steps 0 --rollout-k 32 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --two-streams 0 --envs-per-gpu $NENV > $OUT/bench.log 2>&1 || { echo "pmc pass failed"; tail -5 $OUT/bench.log; exit 1; }
# the fused collect step (cf2_collect_step) on the same workload, from its own per-launch benchmark
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_collect -o pmc -- python3 tools/collect_bench.py --envs $NENV --steps 64 --warmup 300 > $OUT/collect.log 2>&1 || { echo "collect pmc pass failed"; tail -5 $OUT/collect.log; exit 1; }
# the matrix-core side of the fused collect kernel: MFMA-busy cycles (MI355X_MICROARCH.md: counts cycles,
# 16 per v_mfma_f32_16x16x32_bf16), in a pass of its own
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_mfma -o pmc -- python3 tools/collect_bench.py --envs $NENV --steps 64 --warmup 300 > $OUT/collect_mfma.log 2>&1 || { echo "collect mfma pass failed"; tail -5 $OUT/collect_mfma.log; exit 1; }
python3 tools/pmc_valu.py $OUT $NENV
