cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04e
timeout -k 10 120 ./build_ab/dispatch_probe sweep > gpurun_out/r04e/dispatch_sweep.txt 2>&1 || { echo probe failed; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_collect_fused.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r04e/collect_tests.log 2>&1 || { echo "collect tests failed"; tail -40 gpurun_out/r04e/collect_tests.log; exit 1; }
tail -3 gpurun_out/r04e/collect_tests.log
for n in 262144 32768; do timeout -k 10 200 python tools/collect_bench.py --envs $n --steps 256 --warmup 600 >> gpurun_out/r04e/collect_bench.jsonl 2> gpurun_out/r04e/collect_bench.err || { echo "collect bench failed"; tail gpurun_out/r04e/collect_bench.err; exit 1; }; done
cat gpurun_out/r04e/collect_bench.jsonl
bash tools/r04d_session.sh
