cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r04d
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > gpurun_out/r04d/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r04d/pytest.log; exit 1; }
tail -2 gpurun_out/r04d/pytest.log
bash tools/quick_sizes.sh gpurun_out/r04d/sizes.jsonl || exit 1
for n in 4096 32768 262144; do CF2SIM_LIB=build_ab/timing.so timeout -k 10 120 python tools/timeline.py --envs $n --out gpurun_out/r04d/timeline_$n.json > gpurun_out/r04d/timeline_$n.txt 2>&1 || { echo timeline failed; tail gpurun_out/r04d/timeline_$n.txt; exit 1; }; done
CF2_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 300 --warmup 1000 --no-cpu-baseline --weak-envs 0 > gpurun_out/r04d/bench2.json 2> gpurun_out/r04d/bench2.err || { echo "bench2 failed"; tail -20 gpurun_out/r04d/bench2.err; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r04d/bench.json 2> gpurun_out/r04d/bench.err || { echo "bench failed"; tail -20 gpurun_out/r04d/bench.err; exit 1; }
echo done
