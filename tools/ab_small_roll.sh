set -o pipefail
for rep in 1 2; do for lib in build_ab/cur.so build_ab/smallx.so; do
  CF2SIM_LIB=$PWD/$lib timeout -k 10 200 python tools/fused_bench.py 50 2>/dev/null | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$lib rep $rep fused', d['env'][26:], d['N'], round(d['fused_us_per_env_step'],2))" || exit 1
  for cfg in "DroneHoverBulletFreeEnvWithGust-v0 32768" "DroneHoverBulletFreeEnvWithConstWind-v0 4096"; do set -- $cfg
    CF2SIM_LIB=$PWD/$lib timeout -k 10 200 python tools/collect_bench.py --env-id $1 --envs $2 --steps 200 --warmup 1000 2>/dev/null | python -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$lib rep $rep collect', '$1'[26:], $2, 'fused', round(d['fused_us'],2), 'roll', round(d['rollout_us_per_env_step'],2))" || exit 1
  done
done; done
