#!/bin/bash
# Round-3 measurement, part B: the bench line (with the PMC results of part A in profiles/),
# rocprofv3 kernel stats of the timed step launches, the collect loop fused vs two launches and its
# kernel stats.  usage: bash tools/r03_measure_b.sh TAG
set -o pipefail
TAG=${1:-r03b}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o step -- python3 bench.py --steps 1000 --warmup 1000 --no-cpu-baseline --collect-steps 0 --streaming-ring 0 > $OUT/prof_bench.json 2> $OUT/prof.err || { echo "rocprof failed"; tail -20 $OUT/prof.err; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
find $OUT/prof -name "*kernel_trace.csv" | head -1 | xargs -I{} python3 tools/trace_over_time.py {} > $OUT/step_kernel_over_time.txt 2>&1 || true
head -3 $OUT/kernel_stats.csv | cut -c1-160
bash tools/collect_round.sh ${TAG}_collect skip-tests > $OUT/collect.txt 2>&1 || { echo "collect failed"; tail -20 $OUT/collect.txt; exit 1; }
head -2 $OUT/collect.txt
echo done
