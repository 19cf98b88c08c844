set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab2
SKIP_TESTS=1 bash tools/ab_run.sh build_ab/base.so build_ab/cheapreset.so || exit 1
for lib in base cheapreset; do
  for n in 4096 32768; do
    echo "== $lib N=$n"; CF2SIM_LIB=build_ab/$lib.so timeout -k 10 120 python bench.py --steps 200 --warmup 30 --no-cpu-baseline --envs-per-gpu $n --env-id DroneHoverBulletFreeEnvWithGust-v0 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"  kernel {d['roofline']['kernel_ms_per_launch']*1e3:.2f} us\")" || exit 1
  done
done
