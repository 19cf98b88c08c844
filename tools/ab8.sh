set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab8
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/ab8/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/ab8/pytest.log; exit 1; }
tail -2 gpurun_out/ab8/pytest.log
bash tools/ab_rep.sh 3 build_ab/old.so build_ab/new.so 2>&1 | grep rep
for lib in old new; do for n in 4096 32768; do
  CF2SIM_LIB=build_ab/$lib.so timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --rollout-k 0 --envs-per-gpu $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib N=$n', f\"kernel {d['roofline']['kernel_ms_per_launch']*1e3:.2f} us\")" || exit 1
done; done
