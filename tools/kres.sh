#!/bin/bash
# Kernel resource usage (VGPRs / scratch / occupancy) of the gfx950 code object, per kernel.
# usage: tools/kres.sh [extra hipcc flags...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on -fgpu-approx-transcendentals \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I "$ROOT/include" --cuda-device-only -c \
  -Rpass-analysis=kernel-resource-usage "$@" "$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_kernels.hip" \
  -o /tmp/kres.o 2>&1 | python3 -c '
import re,sys
cur=None; rows={}
for l in sys.stdin:
    m=re.search(r"Function Name: (\S+)",l)
    if m: cur=m.group(1); rows[cur]={}; continue
    m=re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|SGPRs): (\d+)",l)
    if m and cur: rows[cur][m.group(1).split()[0]]=m.group(2)
for k,v in rows.items(): print("%-60s V=%s A=%s S=%s occ=%s" % (k[:60], v.get("VGPRs"), v.get("AGPRs"), v.get("ScratchSize"), v.get("Occupancy")))
'
