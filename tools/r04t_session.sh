cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04t && mkdir -p $O
CF2SIM_LIB=build_ab/flag2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_collect_fused.py tests/test_gpu_golden.py tests/test_rollout_fused.py -x -q --timeout 200 --timeout-method thread > $O/flag2_tests.log 2>&1 || { echo "flag2 tests failed"; tail -30 $O/flag2_tests.log; exit 1; }
tail -2 $O/flag2_tests.log
for v in timing_flag timing_flag2; do for n in 4096 32768; do CF2SIM_LIB=build_ab/$v.so timeout -k 10 120 python tools/timeline.py --envs $n --out $O/${v}_$n.json > $O/${v}_$n.txt 2>&1 || { echo timeline failed; tail $O/${v}_$n.txt; exit 1; }; done; done
cat $O/timing_flag_32768.txt $O/timing_flag2_32768.txt
for rep in 1 2; do for v in flag flag2; do bash tools/quick_sizes.sh $O/sizes_${v}_$rep.jsonl build_ab/$v.so > /dev/null || { echo sizes failed; exit 1; }; echo "$v $rep"; cat $O/sizes_${v}_$rep.jsonl; done; done
echo done
