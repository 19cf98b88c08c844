cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04g && mkdir -p $O
for n in 4096 32768; do CF2SIM_LIB=build_ab/timing.so timeout -k 10 120 python tools/timeline.py --envs $n --out $O/timeline_$n.json > $O/timeline_$n.txt 2>&1 || { echo timeline failed; tail $O/timeline_$n.txt; exit 1; }; done
cat $O/timeline_32768.txt
CF2SIM_LIB=build_ab/wsplit.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_collect_fused.py tests/test_gpu_golden.py tests/test_delta_gather_gpu.py -x -q --timeout 200 --timeout-method thread > $O/wsplit_tests.log 2>&1 || { echo "wsplit tests failed"; tail -30 $O/wsplit_tests.log; exit 1; }
tail -2 $O/wsplit_tests.log
for rep in 1 2; do for v in base wsplit; do lib=build_ab/$v.so; [ $v = base ] && lib=""; bash tools/quick_sizes.sh $O/sizes_${v}_$rep.jsonl $lib > /dev/null || { echo sizes failed; exit 1; }; echo "$v $rep"; cat $O/sizes_${v}_$rep.jsonl; done; done
timeout -k 10 170 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
head -c 1500 $O/bench.json
echo done
