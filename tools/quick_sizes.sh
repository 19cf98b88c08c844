#!/bin/bash
# Step-kernel time (HIP events over 2000 launches after 1000 warm-up) of the bench workload at the
# node-shard sizes and at the headline size; one JSON line per size.  usage: tools/quick_sizes.sh OUT [lib]
set -o pipefail
OUT=${1:-gpurun_out/sizes.jsonl}
: > "$OUT"
for n in 4096 32768 262144; do
  CF2SIM_LIB=${2:-} timeout -k 10 200 python bench.py --steps 2000 --warmup 1000 --no-cpu-baseline --collect-steps 0 \
    --rollout-k 32 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --two-streams 0 --envs-per-gpu $n 2>/dev/null |
    python -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'envs': $n, 'kernel_us': d['roofline']['kernel_ms_per_launch']*1e3, 'value': d['value'], 'fused_us': d['fused_rollout']['us_per_env_step']}))" >> "$OUT" || exit 1
done
cat "$OUT"
