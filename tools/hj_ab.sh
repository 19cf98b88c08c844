#!/bin/bash
# A/B of HJ-adversary env-step time across library builds: bash tools/hj_ab.sh lib1.so lib2.so ...
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for env in DroneHoverBulletFreeEnvWithAdversary-v0 DroneHoverBulletFreeEnvWithRandomHJAdversary-v0; do
  for lib in "$@"; do
    CF2SIM_LIB=$lib timeout -k 10 120 python bench.py --steps 100 --warmup 30 --no-cpu-baseline --env-id $env 2>/dev/null |
      python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$env'[:40], '$lib', round(d['roofline']['kernel_ms_per_launch']*1e3,1), 'us')" || exit 1
  done
done
