set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for r in 1 2; do for lib in inplace rec; do for n in 32768 262144; do
  CF2SIM_LIB=build_ab/$lib.so timeout -k 10 120 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --envs-per-gpu $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib N=$n', f\"fused {d['fused_rollout']['us_per_env_step']:.2f} us/env-step\")" || exit 1
done; done; done
