# profiles of the final round-4 kernels: rocprof kernel stats of the default bench, PMC traffic and
# VALU / MFMA passes, the small-N collect loop's kernel stats, timelines at 4096 / 32 768 envs
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04w && mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof bench failed"; tail $O/prof_bench.err; exit 1; }
bash tools/pmc_traffic.sh r04w/traffic 262144 || exit 1
bash tools/pmc_valu.sh r04w/pmc 262144 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_collect_small -o collect -- python3 tools/collect_bench.py --envs 32768 --steps 256 --warmup 600 > $O/prof_collect_small.log 2>&1 || { echo "rocprof collect small failed"; tail $O/prof_collect_small.log; exit 1; }
for n in 4096 32768; do CF2SIM_LIB=build_ab/timing.so timeout -k 10 120 python tools/timeline.py --envs $n --out $O/timeline_$n.json > $O/timeline_$n.txt 2>&1 || { echo timeline failed; tail $O/timeline_$n.txt; exit 1; }; done
echo done
