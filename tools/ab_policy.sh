#!/bin/bash
# A/B the fused policy kernel across library builds: bash tools/ab_policy.sh lib1.so lib2.so ...
set -o pipefail
for lib in "$@"; do
  echo "== $lib"
  CF2SIM_LIB=$lib timeout -k 10 300 python tools/rollout_bench.py --steps 16 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"policy {d['policy_ms_per_step']*1e3:.1f} us/step  env {d['env_ms_per_step']*1e3:.1f} us  rollout {d['rollout_env_steps_per_s']:.3e} env-steps/s\")" || exit 1
done
