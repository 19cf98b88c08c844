#!/bin/bash
# Time the step kernel under feature ablations (env kwargs) to attribute its cost.
set -o pipefail
run() { echo "== $1"; timeout -k 10 300 python bench.py --steps 200 --warmup 30 --no-cpu-baseline --env-kw "$1" $2 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"  {d['roofline']['kernel_ms_per_launch']*1e3:.1f} us/launch  {d['value']:.3e} env-steps/s  {d['roofline']['achieved']:.0f} GB/s (algorithmic {d['roofline']['algorithmic_bytes_per_env_step']} B)\")" || exit 1; }
run '{}'
run '{"observation_noise": 0}'
run '{"domain_randomization": -1}'
run '{"motor_thrust_noise": 0}'
run '{"observation_noise": 0, "domain_randomization": -1, "motor_thrust_noise": 0}'
run '{"max_episode_steps": 0, "enable_reset_distribution": false}'
run '{}' "--env-id DroneHoverBulletFreeEnvWithoutAdversary-v0"
