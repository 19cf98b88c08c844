set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab3
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/ab3/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/ab3/pytest.log; exit 1; }
tail -2 gpurun_out/ab3/pytest.log
SKIP_TESTS=1 bash tools/ab_run.sh build_ab/onewave.so build_ab/roles.so || exit 1
for lib in onewave roles; do
  for n in 4096 32768; do
    echo "== $lib N=$n"; CF2SIM_LIB=build_ab/$lib.so timeout -k 10 120 python bench.py --steps 200 --warmup 30 --no-cpu-baseline --envs-per-gpu $n | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"  kernel {d['roofline']['kernel_ms_per_launch']*1e3:.2f} us\")" || exit 1
  done
done
