#!/bin/bash
# Build an A/B variant of libcf2sim.so into build_ab/NAME.so with extra hipcc flags on the policy
# source (kernels and C-ABI objects reused from the in-tree build).
# usage: tools/build_policy_variant.sh NAME [flags...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
OBJ=$ROOT/disturbance-crazyfile-simulation_amd/cf2sim/_build
mkdir -p "$ROOT/build_ab"
cd /tmp && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=on -fgpu-approx-transcendentals \
  -fno-hip-fp32-correctly-rounded-divide-sqrt ${SLP:--fno-slp-vectorize} -Wall -Wno-pass-failed -I "$ROOT/include" "$@" \
  -c -o "/tmp/pvariant_$name.o" "$ROOT/disturbance-crazyfile-simulation_amd/csrc/cf2sim_policy.hip" &&
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/build_ab/$name.so" "$OBJ/cf2sim_kernels.o" \
  "/tmp/pvariant_$name.o" "$OBJ/cf2sim_util.o" "$OBJ/cf2sim_api.o"
