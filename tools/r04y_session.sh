# the default bench line and the rocprof kernel summary of the same command (round-4 final build)
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04y && mkdir -p $O
timeout -k 10 170 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], json.dumps(d['roofline'])[:500])"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o bench -- python3 bench.py > $O/prof_bench.json 2> $O/prof_bench.err || { echo "rocprof bench failed"; tail $O/prof_bench.err; exit 1; }
head -3 $O/prof/bench_kernel_stats.csv
echo done
