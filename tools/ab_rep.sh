# A/B the step kernel across library builds, R alternating repetitions of 400 steps each:
# bash tools/ab_rep.sh R lib1.so lib2.so ...
set -o pipefail
R=$1; shift
for r in $(seq $R); do for lib in "$@"; do
  CF2SIM_LIB=$lib timeout -k 10 300 python bench.py --steps 400 --warmup 50 --no-cpu-baseline | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(f\"$lib rep $r kernel {d['roofline']['kernel_ms_per_launch']*1e3:.2f} us\")" || exit 1
done; done
