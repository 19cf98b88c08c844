set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in new b128; do for n in 4096 32768 65536 262144; do
  CF2SIM_LIB=build_ab/$lib.so timeout -k 10 120 python bench.py --steps 300 --warmup 30 --no-cpu-baseline --rollout-k 0 --envs-per-gpu $n 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib N=$n', f\"kernel {d['roofline']['kernel_ms_per_launch']*1e3:.2f} us\")" || exit 1
done; done
