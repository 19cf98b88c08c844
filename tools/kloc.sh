#!/bin/bash
# Source lines (file:line) of a given instruction in the main step-kernel variant. usage: tools/kloc.sh REGEX [NOISE DR PHYS]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
pat=$1; n=${2:-1}; d=${3:-1}; p=${4:-0}
b() { [ "$1" = 1 ] && echo Lb1 || echo Lb0; }
K="_ZN3cf211step_kernelI$(b $n)E$(b $d)ELi${p}ELi${SPEC:-1}ELi${ST:-0}EEEvNS_7KParamsENS_6StepIOE"
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -gline-tables-only -std=c++17 -ffp-contract=on -fgpu-approx-transcendentals \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -I "$ROOT/include" --cuda-device-only -S $EXTRA \
  "$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_kernels.hip" -o /tmp/kloc_all.s 2>/dev/null || exit 1
L=$(grep -n "^$K:" /tmp/kloc_all.s | cut -d: -f1)
E=$(grep -n "^.Lfunc_end.*:" /tmp/kloc_all.s | awk -F: -v l=$L '$1>l{print $1; exit}')
sed -n "${L},${E}p" /tmp/kloc_all.s | awk -v pat="$pat" '/\.loc/{f=$2; l=$3} $0 ~ pat {c[f":"l]++} END{for(k in c) print c[k], k}' | sort -rn | head -${TOP:-25}
