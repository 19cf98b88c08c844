# Same-box A/B of two full library builds on the rollout caller (bf16x3 and fp32 policy) and the
# step() bench at action rings 8 and 64.  usage: bash tools/ab_rollout_nt.sh LIB_A LIB_B (builds: tools/build_variant.sh)
set -o pipefail
for rep in 1 2; do for lib in "$@"; do
  for p in bf16x3 fp32; do
    CF2SIM_LIB=$lib timeout -k 10 200 python tools/rollout_bench.py --precision $p 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib rep $rep $p rollout', round(d['ms_per_step']*1e3,1), 'us/step, policy alone', round(d['policy_ms_per_step']*1e3,1))" || exit 1
  done
  for R in 8 64; do
    CF2SIM_LIB=$lib timeout -k 10 120 python bench.py --steps 2000 --warmup 1000 --no-cpu-baseline --rollout-k 0 --streaming-ring 0 --action-ring $R 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib rep $rep ring $R step', round(d['roofline']['kernel_ms_per_launch']*1e3,2))" || exit 1
  done
done; done
