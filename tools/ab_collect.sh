#!/bin/bash
# A/B of the fused collect step across library builds (build_ab/*.so from tools/build_variant.sh):
# collect env-steps at 262 144 envs, bf16x3, R alternating repetitions.  usage: ab_collect.sh R lib...
set -o pipefail
R=$1; shift
for r in $(seq $R); do for lib in "$@"; do
  CF2SIM_LIB=$lib timeout -k 10 200 python tools/rollout_bench.py --precision bf16x3 --env-warmup 300 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"$lib rep $r collect {d['ms_per_step']*1e3:.2f} us/env-step\")" || exit 1
done; done
