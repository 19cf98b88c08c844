#!/bin/bash
# Fused collect step (cf2_collect_step) on one MI355X: parity tests, collect throughput fused vs two
# launches per step at 262 144 envs (bf16x3), rocprofv3 kernel stats of the fused collect.
# usage: bash tools/collect_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-collect}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_collect_fused.py tests/test_rollout.py tests/test_rollout_reference.py \
    -x -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { echo "tests failed"; tail -40 $OUT/tests.log; exit 1; }
  tail -3 $OUT/tests.log
fi
for v in fused unfused; do
  extra=""; [ $v = unfused ] && extra="--no-fuse"
  timeout -k 10 200 python tools/rollout_bench.py --precision bf16x3 $extra > $OUT/rollout_$v.json 2> $OUT/rollout_$v.err || { tail -5 $OUT/rollout_$v.err; exit 1; }
  cat $OUT/rollout_$v.json
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o r -- python3 tools/rollout_bench.py --precision bf16x3 > /dev/null 2> $OUT/prof.err || { tail -5 $OUT/prof.err; exit 1; }
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats.csv
cut -d, -f1-4 $OUT/kernel_stats.csv | cut -c1-150 | head -12
