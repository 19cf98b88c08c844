# rollout caller at 262144 envs: per-kernel rocprof stats, both policy precisions. usage: rollout_prof.sh TAG
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-rprof}; mkdir -p $OUT
for p in fp32 bf16x3; do
  timeout -k 10 120 python tools/rollout_bench.py --precision $p > $OUT/rollout_$p.json 2> $OUT/rollout_$p.err || { tail -5 $OUT/rollout_$p.err; exit 1; }
  cat $OUT/rollout_$p.json
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$p -o r -- python3 tools/rollout_bench.py --precision $p > /dev/null 2> $OUT/prof_$p.err || { tail -5 $OUT/prof_$p.err; exit 1; }
  f=$(find $OUT/prof_$p -name "*kernel_stats.csv" | head -1); cp $f $OUT/kernel_stats_$p.csv
  f=$(find $OUT/prof_$p -name "*kernel_trace.csv" | head -1); python tools/kernel_gaps.py $f > $OUT/gaps_$p.txt; cat $OUT/gaps_$p.txt
  cut -d, -f1-4 $OUT/kernel_stats_$p.csv | cut -c1-150 | head -12
done
# time-out-heavy collect (TimeLimit 40 steps: ~2.5 % of the envs time out per step)
timeout -k 10 120 python tools/rollout_bench.py --precision bf16x3 --max-episode-steps 40 > $OUT/rollout_bf16x3_tl40.json 2> $OUT/rollout_tl40.err || { tail -5 $OUT/rollout_tl40.err; exit 1; }
cat $OUT/rollout_bf16x3_tl40.json
