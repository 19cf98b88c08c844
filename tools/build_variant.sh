#!/bin/bash
# Build an A/B variant of libcf2sim.so into build_ab/NAME.so with extra hipcc flags.
# usage: [CF2_FULL=1] [KSRC=other_kernels.hip] tools/build_variant.sh NAME [flags...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
KSRC=${KSRC:-$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_kernels.hip}
mkdir -p "$ROOT/build_ab"
# only the bench workload's kernel instance unless CF2_FULL=1 (a variant then builds in ~1/8 the time)
ONLY=-DCF2_BENCH_ONLY; [ -n "$CF2_FULL" ] && ONLY=
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -ffp-contract=fast -fgpu-approx-transcendentals \
  -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-slp-vectorize -Wall -Wno-pass-failed -I "$ROOT/include" \
  -I "$ROOT/disturbance-crazyfile-simulation_amd/csrc" $ONLY "$@" -o "$ROOT/build_ab/$name.so" \
  "$KSRC" "$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_policy.hip" \
  "$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_api.cpp"
