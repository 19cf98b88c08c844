#!/bin/bash
# A/B step-kernel time of library builds at several env counts and env ids.
# usage: bash tools/ab_envs.sh "ENV_ID:N ENV_ID:N ..." lib1.so lib2.so ...
set -o pipefail
cases=$1; shift
for r in 1 2 3; do for c in $cases; do for lib in "$@"; do
  id=${c%%:*}; n=${c##*:}
  CF2SIM_LIB=$lib timeout -k 10 120 python bench.py --steps 1000 --warmup 1000 --no-cpu-baseline --rollout-k 0 --streaming-ring 0 --oc-envs 0 --env-id $id --envs-per-gpu $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"$lib $id N=$n kernel {d['roofline']['kernel_ms_per_launch']*1e3:.2f} us\")" || exit 1
done; done; done
