#!/bin/bash
# One bench line per BASELINE.json config on one GPU (C1 is the CPU oracle: bench.py's cpu_baseline),
# plus the HJ-adversary env (f1) on synthetic value tables.  usage: bash tools/all_configs.sh [OUT]
set -o pipefail
OUT=${1:-gpurun_out/all_configs.jsonl}
cd "$GRAFT_REPO_ROOT"
: > "$OUT"
: > "$OUT.err"
run() {   # label, bench args...
  local label=$1; shift
  timeout -k 10 180 python bench.py --steps 2000 --warmup 1000 --no-cpu-baseline --rollout-k 32 --streaming-ring 0 --oc-envs 0 "$@" 2>>"$OUT.err" |
    python -c "import json,sys; d=json.loads(sys.stdin.read()); d['label']='$label'; print(json.dumps(d))" >> "$OUT" || exit 1
}
run C2 --env-id DroneHoverBulletFreeEnvWithConstWind-v0 --envs-per-gpu 4096
run C3 --env-id DroneHoverBulletFreeEnvWithRandomAdversary-v0 --envs-per-gpu 65536
run C4-shard --env-id DroneHoverBulletFreeEnvWithGust-v0 --envs-per-gpu 32768
run C4 --env-id DroneHoverBulletFreeEnvWithGust-v0 --envs-per-gpu 262144
run C5 --env-id DroneHoverBulletFreeEnvWithDownwash-v0 --envs-per-gpu 262144
run HJ --env-id DroneHoverBulletFreeEnvWithAdversary-v0 --envs-per-gpu 262144
run HJ-Boltzmann --env-id DroneHoverBulletFreeEnvWithRandomHJAdversary-v0 --envs-per-gpu 262144
python - "$OUT" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    r = d["roofline"]
    print(f"{d['label']:13s} {d['config']['envs_per_gpu']:7d} envs  {d['value']:.3e} env-steps/s  "
          f"kernel {r['kernel_ms_per_launch'] * 1e3:6.1f} us  {r['achieved']:6.0f} GB/s  fused {d['fused_rollout']['us_per_env_step']:6.1f} us/env-step")
PY
