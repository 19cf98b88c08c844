cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && O=gpurun_out/r04v && mkdir -p $O
CF2SIM_LIB=build_ab/roll_flag.so timeout -k 10 400 python -u -m pytest tests/test_rollout_fused.py tests/test_collect_fused.py tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo "roll_flag tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for rep in 1 2; do for v in flag2 roll_flag; do
for n in 4096 32768; do CF2SIM_LIB=build_ab/$v.so timeout -k 10 200 python tools/collect_bench.py --envs $n --steps 256 --warmup 600 2>/dev/null | sed "s/^/$v $rep /" >> $O/collect_ab.txt || { echo collect ab failed; exit 1; }; done
bash tools/quick_sizes.sh $O/sizes_${v}_$rep.jsonl build_ab/$v.so > /dev/null || { echo sizes failed; exit 1; }; echo "$v $rep"; cat $O/sizes_${v}_$rep.jsonl
done; done
cut -c1-400 $O/collect_ab.txt
echo done
