#!/bin/bash
# Where the step kernel's VGPR pressure peaks: max VGPR index per 100 ISA lines (spill lanes
# excluded), plus markers for the phase fences.  usage: tools/vprof.sh [hipcc -D flags]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on -fgpu-approx-transcendentals \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I "$ROOT/include" --cuda-device-only -S "$@" \
  "$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_kernels.hip" -o /tmp/vprof_all.s 2>/dev/null || exit 1
awk '/^_ZN3cf211step_kernel/,/s_endpgm/' /tmp/vprof_all.s > /tmp/vprof.s
python3 - <<'PY'
import re
L=open('/tmp/vprof.s').read().split('\n')
out=[]
for c in range(0,len(L),100):
    mx=-1; fence=False
    for l in L[c:c+100]:
        if 'sched_barrier' in l: fence=True
        if 'readlane' in l or 'writelane' in l: continue
        for m in re.finditer(r'v\[(\d+):(\d+)\]|\bv(\d+)\b', l):
            mx=max(mx,int(m.group(2) or m.group(3)))
    out.append(f"{c}:{mx}{'|' if fence else ''}")
print(' '.join(out))
PY
