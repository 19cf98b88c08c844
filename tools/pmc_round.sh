#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per pass, as the gfx950 PMC
# slot table requires: FETCH_SIZE and WRITE_SIZE never share a pass).  usage: pmc_round.sh TAG [bench args]
set -o pipefail
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--steps 30 --warmup 5 --no-cpu-baseline $*"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "GRBM_GUI_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 $OUT/p$i.log; }
done
python3 tools/pmc_parse.py $OUT
