"""In-tree build of libcf2sim.so with hipcc for gfx950 (no JIT cache: the .so travels with the repo)."""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
SRC_DIR = os.path.abspath(os.path.join(PKG_DIR, "..", "csrc"))
INC_DIR = os.path.abspath(os.path.join(PKG_DIR, "..", "..", "include"))
LIB = os.path.join(PKG_DIR, "libcf2sim.so")
SOURCES = ["cf2sim_kernels.hip", "cf2sim_policy.hip", "cf2sim_util.hip", "cf2sim_exchange.hip", "cf2sim_api.cpp"]
HEADERS = ["cf2sim_internal.h", "cf2sim_rng.h", "cf2sim_policy.h", "cf2sim_pack.h"]
# The env-step is fp32 throughout.  FMA contraction, approximate division/sqrt (v_rcp / v_sqrt,
# ~1 ulp) and the hardware sin/cos/log are allowed: the kernel is compared against the fp32 and
# fp64 CPU restatements with stated tolerances (tests/test_gpu_parity.py), not bitwise.
FLAGS = ["--offload-arch=gfx950", "-O3", "-fPIC", "-shared", "-std=c++17", "-ffp-contract=fast",
         "-fgpu-approx-transcendentals", "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-pass-failed"]
# per-source extras: no SLP vectorisation (packed v_pk_* f32 ops need register-pair shuffles
# that cost more than they save in the env-step kernels: +3 us).  The policy kernel gained 2 us
# from SLP at 2 waves/SIMD, but at its current 4 waves/SIMD shape SLP makes it spill (56 B/lane,
# bf16x3 40.0 us vs 38.3 us without)
# The env kernels contract a*b+c only within one source expression (-ffp-contract=on, after the
# global fast): with "fast" the backend also fused across statements wherever the surrounding code
# allowed, so the small-N and the large-N step kernels rounded some sums differently (gyro bias,
# reset pose: 1-ulp differences, then chaotic growth) and a run's results depended on the envs per
# context, i.e. on the rank count.  "on" makes every launch geometry bit-identical
# (tests/test_gpu_fullsize.py, contexts of 131 072 / 65 536 / 2 x 32 768 against one of 262 144) at
# no measured cost (262 144 envs 36.08-36.19 vs 36.06-36.13 us, 32 768 envs within noise).
SOURCE_FLAGS = {"cf2sim_kernels.hip": ["-fno-slp-vectorize", "-ffp-contract=on"], "cf2sim_api.cpp": ["-fno-slp-vectorize"],
                "cf2sim_policy.hip": ["-fno-slp-vectorize", "-ffp-contract=on"]}
# The policy TU contracts like the env kernels too: the fused collect kernel (cf2sim_kernels.hip)
# runs the same policy code (cf2sim_policy.h), and with "fast" the policy kernel alone fused the
# standardisation's product into the hi/lo split's subtraction (8 v_fma instead of v_sub), so the
# two paths' actions and values differed in the last bit in ~20 % of rows.


def _hipcc() -> str:
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        raise RuntimeError("hipcc not found")
    return h


BUILD_DIR = os.path.join(PKG_DIR, "_build")

# -D defines the native sources know.  CF2_TIMING adds the per-wave phase stamps tools/timeline.py
# reads (cf2_debug_timing_buffer); it changes no result.  Any other CF2_ define is a typo or a
# removed A/B knob: it would compile silently into a library that differs from the tested one, so
# it is rejected.
KNOWN_DEFINES = frozenset({"CF2_TIMING"})


def check_defines(flags) -> None:
    """ValueError for a -DCF2_* flag that is not in KNOWN_DEFINES."""
    for f in flags:
        if not f.startswith("-D"):
            continue
        name = f[2:].split("=", 1)[0]
        if name.startswith("CF2_") and name not in KNOWN_DEFINES:
            raise ValueError(f"unknown define {name}: the native sources only know {sorted(KNOWN_DEFINES)}")


def _digest(*parts: bytes) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(p)
        h.update(b"\0")
    return h.hexdigest()


def _read(path: str) -> bytes:
    with open(path, "rb") as f:
        return f.read()


def _headers_blob() -> bytes:
    return b"".join(_read(os.path.join(SRC_DIR, h)) for h in HEADERS) + _read(os.path.join(INC_DIR, "cf2sim.h"))


def _compile_flags(src: str | None = None, extra=()):
    return [f for f in FLAGS if f != "-shared"] + SOURCE_FLAGS.get(src, []) + list(extra) + ["-c"]


def _obj_key(src: str, extra=()) -> str:
    return _digest(" ".join(_compile_flags(src, extra)).encode(), _read(os.path.join(SRC_DIR, src)), _headers_blob())


def _lib_key(extra=()) -> str:
    return _digest(*[_obj_key(s, extra).encode() for s in SOURCES])


def _stamp(path: str) -> str | None:
    try:
        with open(path + ".stamp") as f:
            return f.read().strip()
    except OSError:
        return None


def up_to_date() -> bool:
    """Content-addressed (sources, headers, flags), not mtime-based: a copied tree (e.g. the GPU
    box snapshot) with an already built library does not rebuild."""
    return os.path.exists(LIB) and _stamp(LIB) == _lib_key()


def build_native(force: bool = False, verbose: bool = False, extra_flags=(), out: str | None = None) -> str:
    """Build libcf2sim.so in-tree (or, with extra_flags, e.g. ['-DCF2_TIMING'], a variant at `out`,
    from objects in their own build directory, leaving the in-tree library untouched)."""
    extra = list(extra_flags)
    check_defines(extra)
    if extra and out is None:
        raise ValueError("a build with extra flags needs an output path (out=): the in-tree library is the tested one")
    lib = os.path.abspath(out) if out else LIB
    bdir = BUILD_DIR if not extra else BUILD_DIR + "_" + _digest(" ".join(extra).encode())[:12]
    if not force and os.path.exists(lib) and _stamp(lib) == _lib_key(extra):
        return lib
    os.makedirs(bdir, exist_ok=True)
    os.makedirs(os.path.dirname(lib), exist_ok=True)
    procs = []
    objs = []
    for src in SOURCES:      # one object per source, compiled in parallel, skipped when unchanged
        obj = os.path.join(bdir, os.path.splitext(src)[0] + ".o")
        objs.append(obj)
        key = _obj_key(src, extra)
        if not force and os.path.exists(obj) and _stamp(obj) == key:
            continue
        cmd = [_hipcc(), *_compile_flags(src, extra), "-I", INC_DIR, "-o", obj + ".tmp", os.path.join(SRC_DIR, src)]
        if verbose:
            print(" ".join(cmd))
        procs.append((subprocess.Popen(cmd), obj, key))
    failed = False
    for p, obj, key in procs:
        if p.wait() != 0:
            failed = True
            continue
        os.replace(obj + ".tmp", obj)
        with open(obj + ".stamp", "w") as f:
            f.write(key)
    if failed:
        raise subprocess.CalledProcessError(1, "hipcc")
    cmd = [_hipcc(), "--offload-arch=gfx950", "-shared", "-fPIC", "-o", lib + ".tmp", *objs]
    if verbose:
        print(" ".join(cmd))
    subprocess.run(cmd, check=True)
    os.replace(lib + ".tmp", lib)
    with open(lib + ".stamp", "w") as f:
        f.write(_lib_key(extra))
    return lib
