"""In-tree build of libcf2sim.so with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import os
import shutil
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC_DIR = os.path.abspath(os.path.join(PKG_DIR, "..", "csrc"))
INC_DIR = os.path.abspath(os.path.join(PKG_DIR, "..", "..", "include"))
LIB = os.path.join(PKG_DIR, "libcf2sim.so")
SOURCES = ["cf2sim_kernels.hip", "cf2sim_policy.hip", "cf2sim_api.cpp"]
HEADERS = ["cf2sim_internal.h", "cf2sim_rng.h"]
# The env-step is fp32 throughout.  FMA contraction, approximate division/sqrt (v_rcp / v_sqrt,
# ~1 ulp) and the hardware sin/cos/log are allowed: the kernel is compared against the fp32 and
# fp64 CPU restatements with stated tolerances (tests/test_gpu_parity.py), not bitwise.
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=fast",
         "-fgpu-approx-transcendentals", "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-pass-failed",
         "-fno-slp-vectorize"]   # SLP-packed v_pk_* f32 ops need register-pair shuffles that cost more than they save


def _hipcc() -> str:
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        raise RuntimeError("hipcc not found")
    return h


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    deps = [os.path.join(SRC_DIR, s) for s in SOURCES + HEADERS] + [os.path.join(INC_DIR, "cf2sim.h")]
    return all(os.path.getmtime(d) <= t for d in deps)


def build_native(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    cmd = [_hipcc(), *FLAGS, "-I", INC_DIR, "-o", LIB + ".tmp", *[os.path.join(SRC_DIR, s) for s in SOURCES]]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(LIB + ".tmp", LIB)
    return LIB
