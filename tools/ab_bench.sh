#!/bin/bash
# A/B the step kernel across library builds: bash tools/ab_bench.sh lib1.so lib2.so ...
set -o pipefail
for lib in "$@"; do
  echo "== $lib"
  CF2SIM_LIB=$lib timeout -k 10 300 python bench.py --steps 200 --warmup 30 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"value {d['value']:.4e} env-steps/s  kernel {d['roofline']['kernel_ms_per_launch']*1e3:.1f} us  {d['roofline']['achieved']:.0f} GB/s  frac {d['roofline']['frac']:.3f}\")" || exit 1
done
