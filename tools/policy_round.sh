# GPU: rollout/policy tests, then the rollout bench (policy vs env split)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${1:-pol}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_rollout.py tests/test_rollout_fused.py tests/test_rollout_reference.py -q -m gpu -x -s --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python tools/rollout_bench.py > $OUT/rollout.json 2> $OUT/rollout.err || { echo "rollout bench failed"; tail -20 $OUT/rollout.err; exit 1; }
cat $OUT/rollout.json
