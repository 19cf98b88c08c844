set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab7
timeout -k 10 600 python -u -m pytest tests/test_rollout_fused.py tests/test_gpu_parity.py -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/ab7/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/ab7/pytest.log; exit 1; }
tail -2 gpurun_out/ab7/pytest.log
for lib in rcur rroles; do for n in 32768 262144; do
  CF2SIM_LIB=build_ab/$lib.so timeout -k 10 120 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --envs-per-gpu $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib N=$n', f\"step {d['roofline']['kernel_ms_per_launch']*1e3:.2f} us  fused {d['fused_rollout']['us_per_env_step']:.2f} us/env-step\")" || exit 1
done; done
