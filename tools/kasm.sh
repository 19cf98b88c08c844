#!/bin/bash
# ISA of one step-kernel variant + instruction histogram.  usage: tools/kasm.sh [NOISE DR PHYS] (default 1 1 0)
ROOT=$(cd "$(dirname "$0")/.." && pwd)
n=${1:-1}; d=${2:-1}; p=${3:-0}
b() { [ "$1" = 1 ] && echo Lb1 || echo Lb0; }
K="_ZN3cf211step_kernelI$(b $n)E$(b $d)ELi${p}ELi${SPEC:-1}EEEvNS_7KParamsENS_6StepIOE"
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=on -fgpu-approx-transcendentals \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I "$ROOT/include" --cuda-device-only -S $EXTRA \
  "$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_kernels.hip" -o /tmp/kasm_all.s 2>/dev/null || exit 1
L=$(grep -n "^$K:" /tmp/kasm_all.s | cut -d: -f1)
E=$(grep -n "^.Lfunc_end.*:" /tmp/kasm_all.s | awk -F: -v l=$L '$1>l{print $1; exit}')
sed -n "${L},${E}p" /tmp/kasm_all.s > /tmp/kasm.s
echo "VALU static: $(grep -cP '^\s+v_' /tmp/kasm.s)  readlane: $(grep -c v_readlane /tmp/kasm.s)  writelane: $(grep -c v_writelane /tmp/kasm.s)  SALU: $(grep -cP '^\s+s_(?!waitcnt|nop|cbranch|branch)' /tmp/kasm.s)"
grep -oP "^\s+\K[vs]_[a-z0-9_]+" /tmp/kasm.s | sort | uniq -c | sort -rn | head -${TOP:-25}
