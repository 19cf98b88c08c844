cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04f && mkdir -p $O
for n in 4096 32768 262144; do CF2SIM_LIB=build_ab/timing.so timeout -k 10 120 python tools/timeline.py --envs $n --out $O/timeline_$n.json > $O/timeline_$n.txt 2>&1 || { echo timeline failed; tail $O/timeline_$n.txt; exit 1; }; done
for rep in 1; do for v in cr_base cr_xbatch cr_pref; do CF2SIM_LIB=build_ab/$v.so timeout -k 10 200 python tools/collect_bench.py --envs 262144 --steps 256 --warmup 600 | sed "s/^/$v /" >> $O/collect_ab.txt || { echo collect ab failed; exit 1; }; done; done
cat $O/collect_ab.txt
timeout -k 10 300 python tools/collect_streams_bench.py --envs 262144 --steps 32 --splits 1,2,4 > $O/streams.jsonl 2> $O/streams.err || { echo streams failed; tail $O/streams.err; exit 1; }
cat $O/streams.jsonl
for rep in 1 2; do for v in base envrows; do lib=build_ab/$v.so; [ $v = base ] && lib=""; bash tools/quick_sizes.sh $O/sizes_${v}_$rep.jsonl $lib > /dev/null || { echo sizes failed; exit 1; }; done; done
tail -n +1 $O/sizes_*.jsonl
CF2SIM_LIB=build_ab/envrows.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_collect_fused.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > $O/envrows_tests.log 2>&1 || { echo "envrows tests failed"; tail -30 $O/envrows_tests.log; exit 1; }
tail -2 $O/envrows_tests.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_collect -o collect -- python3 tools/collect_bench.py --envs 262144 --steps 256 --warmup 600 > $O/prof_collect.log 2>&1 || { echo "rocprof collect failed"; tail $O/prof_collect.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_collect_small -o collect -- python3 tools/collect_bench.py --envs 32768 --steps 256 --warmup 600 > $O/prof_collect_small.log 2>&1 || { echo "rocprof collect small failed"; tail $O/prof_collect_small.log; exit 1; }
bash tools/pmc_valu.sh r04f/pmc 262144 || exit 1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json | head -c 3000
echo done
