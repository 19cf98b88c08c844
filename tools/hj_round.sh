set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/hj
timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -k "hj or HJ or Adversary or fused or golden or rollout or policy" --timeout 120 --timeout-method thread > gpurun_out/hj/pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/hj/pytest.log; exit 1; }
tail -2 gpurun_out/hj/pytest.log
for e in DroneHoverBulletFreeEnvWithAdversary-v0 DroneHoverBulletFreeEnvWithRandomHJAdversary-v0; do
  timeout -k 10 200 python bench.py --env-id $e --no-cpu-baseline --rollout-k 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$e', f\"{d['value']:.3e} kernel {d['roofline']['kernel_ms_per_launch']*1e3:.2f} us\")" || exit 1
done
