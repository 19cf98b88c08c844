#!/bin/bash
# A/B of the fused collect step's per-launch time (tools/collect_bench.py) across library builds,
# R alternating repetitions.  usage: ab_collect2.sh R lib...
set -o pipefail
R=$1; shift
for r in $(seq $R); do for lib in "$@"; do
  CF2SIM_LIB=$lib timeout -k 10 200 python tools/collect_bench.py --warmup ${WARMUP:-600} | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"$lib rep $r fused {d['fused_us']:.2f} / {d['fused_us_again']:.2f} us, two launches {d['two_launch_us']:.2f} us\")" || exit 1
done; done
