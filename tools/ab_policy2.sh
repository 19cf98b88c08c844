# fused policy forward alone (tools/policy_bench.py) across library builds and precisions
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in "$@"; do for p in bf16x3 fp32; do
  CF2SIM_LIB=$lib timeout -k 10 120 python tools/policy_bench.py --precision $p 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib $p', f\"{d['us_per_forward']:.1f} us\")" || exit 1
done; done
