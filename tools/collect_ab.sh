# A/B of the collect loop between the in-tree library and variant builds (CF2SIM_LIB), alternating
# usage: bash tools/collect_ab.sh OUTDIR variant.so...
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
for rep in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then unset CF2SIM_LIB; else export CF2SIM_LIB=$PWD/$v; fi
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --rollout-k 0 --streaming-ring 0 --oc-envs 0 --exchange-probe 0 --collect-steps 64 > $OUT/c.json 2> $OUT/c.err || { tail -5 $OUT/c.err; exit 1; }
    python -c "import json,sys; d=json.loads(open('$OUT/c.json').read().strip().splitlines()[-1]); c=d['collect']; print('$v', round(c['us_per_env_step'],2), round(c.get('us_per_env_step_one_launch_per_step') or 0,2))"
  done
done
