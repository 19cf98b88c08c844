set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in 32768 4096 65536; do
  CF2SIM_LIB=build_ab/timing.so timeout -k 10 120 python tools/timeline.py --envs $n --warmup 1000 > $O/timeline_$n.txt 2>&1 || { echo "timeline $n failed"; tail -20 $O/timeline_$n.txt; exit 1; }
  grep -v "reset waves\|role-2\|amdgpu.ids" $O/timeline_$n.txt
done
