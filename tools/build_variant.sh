#!/bin/bash
# Build an A/B variant of libcf2sim.so into build_ab/NAME.so with extra hipcc flags on the kernel
# source and the C-ABI (both see the internal KParams layout); the policy object is reused from
# the in-tree build (cf2sim/_build).
# usage: [CF2_FULL=1] [KSRC=other_kernels.hip] [KFLAGS="kernel-only flags"] tools/build_variant.sh NAME [flags...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
KSRC=${KSRC:-$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_kernels.hip}
OBJ=$ROOT/disturbance-crazyfile-simulation_amd/cf2sim/_build
mkdir -p "$ROOT/build_ab"
# only the bench workload's kernel instance unless CF2_FULL=1
ONLY=-DCF2_BENCH_ONLY; [ -n "$CF2_FULL" ] && ONLY=
[ -f "$OBJ/cf2sim_policy.o" ] || { echo "build the in-tree library first"; exit 1; }
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=on -fgpu-approx-transcendentals \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -Wall -Wno-pass-failed -Wno-unused-function -I "$ROOT/include" \
  -I "$ROOT/disturbance-crazyfile-simulation_amd/csrc" $ONLY $KFLAGS "$@" -c -o "/tmp/variant_$name.o" "$KSRC" &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -I "$ROOT/include" "$@" -c -o "/tmp/variant_api_$name.o" \
  "$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_api.cpp" &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/build_ab/$name.so" "/tmp/variant_$name.o" \
  "$OBJ/cf2sim_policy.o" "$OBJ/cf2sim_util.o" "/tmp/variant_api_$name.o"
