#!/bin/bash
# Step-kernel time vs env count (wave-latency vs throughput regime).  usage: tools/nscale.sh [lib]
set -o pipefail
for n in 16384 65536 131072 196608 262144 393216 524288 1048576; do
  CF2SIM_LIB=${1:-} timeout -k 10 300 python bench.py --steps 100 --warmup 20 --no-cpu-baseline --envs-per-gpu $n | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(f\"N={$n:8d}  kernel {r['kernel_ms_per_launch']*1e3:7.1f} us  {d['value']:.3e} env-steps/s  {r['achieved']:.0f} GB/s\")" || exit 1
done
