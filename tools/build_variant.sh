#!/bin/bash
# Build a variant of libcf2sim.so into build_ab/NAME.so with extra hipcc flags on every source,
# through cf2sim.build (which rejects -DCF2_* defines the sources do not know; the only one is
# CF2_TIMING, the phase stamps of tools/timeline.py).  Variants of the kernel source itself are
# kept as patches and applied to a copy of the tree.
# usage: tools/build_variant.sh NAME [flags...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
python3 - "$ROOT" "$name" "$@" <<'PY'
import os, sys
root, name, flags = sys.argv[1], sys.argv[2], sys.argv[3:]
sys.path.insert(0, os.path.join(root, "disturbance-crazyfile-simulation_amd"))
from cf2sim.build import build_native
print(build_native(extra_flags=flags, out=os.path.join(root, "build_ab", name + ".so")))
PY
