"""C-ABI checks that need no GPU: libcf2sim.so loads, exports every entry point that
include/cf2sim.h declares, its cf2_config matches the Python mirror, and error paths return
status codes instead of aborting."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cf2sim.h")


def declared_functions():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char\*)\s+(cf2_\w+)\s*\(", txt, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from cf2sim.build import build_native
    build_native()
    from cf2sim import _native
    return _native.load()


def test_header_declares_expected_entry_points():
    from cf2sim._native import EXPORTED_SYMBOLS
    assert declared_functions() == sorted(EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(lib):
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = os.popen(f"nm -D --defined-only {lib._name}").read()
    for name in declared_functions():
        assert re.search(rf"\bT {name}\b", out), f"{name} not exported"


def test_config_struct_matches(lib):
    from cf2sim.config import CF2Config
    assert lib.cf2_config_sizeof() == ctypes.sizeof(CF2Config)
    assert lib.cf2_abi_version() == 8


def test_status_strings_and_invalid_args(lib):
    from cf2sim.config import build_config
    assert lib.cf2_status_string(0) == b"ok"
    assert lib.cf2_status_string(-5).startswith(b"HJ disturbance")
    ctx = ctypes.c_void_p()
    assert lib.cf2_create(None, ctypes.byref(ctx)) == -1
    bad = build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", 4)
    bad.num_envs = 0
    assert lib.cf2_create(ctypes.byref(bad), ctypes.byref(ctx)) == -1
    bad = build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", 4)
    bad.aggregate_phy_steps = 9
    assert lib.cf2_create(ctypes.byref(bad), ctypes.byref(ctx)) == -4
    assert lib.cf2_destroy(None) == -1
    assert lib.cf2_step(None, None, None, None, None, None, None, None, None, None, None) == -1
    assert lib.cf2_reset(None, None, None, None) == -1


def test_config_constants_match_reference_env_config_dump():
    """Values the reference's own run dumped (train_results_phoenix/.../env_config.json,
    copied as data into tests/golden/env_config_excerpt.json)."""
    import json
    from cf2sim.config import build_config
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "env_config_excerpt.json")))
    c = build_config("DroneHoverBulletFreeEnvWithoutAdversary-v0", 1)
    assert abs(c.K - ref["K"]) < 1e-15
    assert abs(c.A - ref["A"]) < 1e-15 and abs(c.B - ref["B"]) < 1e-15
    assert abs(c.hover_x - ref["HOVER_X"]) < 1e-15
    assert abs(c.hover_action - ref["HOVER_ACTION"]) < 1e-15
    assert c.buf_size == ref["buf_size"]
    assert (c.ixx, c.iyy, c.izz) == tuple(ref["J_diag"])
    assert c.mass == ref["M"] and c.drag_xy == ref["DRAG_COEFF"][0] and c.drag_z == ref["DRAG_COEFF"][2]
    assert c.time_step == ref["TIME_STEP"] and c.obs_rate == 2 and c.aggregate_phy_steps == 2
    assert c.domain_randomization == ref["domain_randomization"]
    assert c.motor_thrust_noise == ref["motor_thrust_noise"]


def test_registry_covers_reference_hover_ids():
    from cf2sim.config import OUT_OF_SCOPE_IDS, REFERENCE_IDS, spec_for_id
    # phoenix_drone_simulation/__init__.py registers 15 ids: 11 hover ids (this path) + 4 take-off/circle
    assert len(REFERENCE_IDS) == 11
    for i in REFERENCE_IDS:
        assert spec_for_id(i).registered_id == i
    for i in OUT_OF_SCOPE_IDS:
        with pytest.raises(NotImplementedError):
            spec_for_id(i)


def test_build_rejects_unknown_defines():
    """cf2sim.build refuses -DCF2_* defines the sources do not know (a removed A/B knob or a typo
    would otherwise compile silently into a library that differs from the tested one)."""
    import pytest
    from cf2sim.build import check_defines, build_native
    check_defines(["-DCF2_TIMING", "-O2", "-DNDEBUG"])
    for bad in (["-DCF2_AB_NO_RESET"], ["-DCF2_SMALL_OLD=1"], ["-DCF2_TIMNG"]):
        with pytest.raises(ValueError):
            check_defines(bad)
        with pytest.raises(ValueError):
            build_native(extra_flags=bad, out="/tmp/never_built.so")
    with pytest.raises(ValueError):           # extra flags never overwrite the in-tree library
        build_native(extra_flags=["-DCF2_TIMING"])


def test_kernel_sources_hold_no_ab_branches():
    """The only preprocessor conditional in the native sources is CF2_TIMING."""
    import glob
    import re
    src = os.path.join(ROOT, "disturbance-crazyfile-simulation_amd", "csrc")
    for f in glob.glob(os.path.join(src, "*")):
        for line in open(f):
            m = re.match(r"\s*#\s*(if|ifdef|ifndef|elif)\b(.*)", line)
            if m:
                assert "CF2_TIMING" in m.group(2), f"{os.path.basename(f)}: {line.strip()}"


def test_obs_exchange_error_paths(lib):
    """cf2_obs_pack / cf2_obs_consume / cf2_obs_rows / cf2_xchg_* reject bad sizes and pointers
    without launching anything (no GPU needed)."""
    from cf2sim.dist import packed_words
    assert lib.cf2_obs_packed_words(32768, 13, 2458) == packed_words(32768, 13, 2458)
    assert lib.cf2_obs_packed_words(5, 17, 3) == packed_words(5, 17, 3)
    assert lib.cf2_obs_packed_words(0, 13, 0) == 0 and lib.cf2_obs_packed_words(8, 12, 1) == 0
    assert lib.cf2_obs_packed_words(8, 13, 9) == 0                      # cap > n
    assert lib.cf2_obs_pack(None, None, 8, 13, 1, None, None, None, None) == -1
    assert lib.cf2_step_packed(*([None] * 10), 1, None) == -1
    w = lib.cf2_obs_packed_words(32768, 13, 32768)
    assert lib.cf2_xchg_send_words(32768, 13, 2, 16) == 2 * 16 * (w + 32)
    assert lib.cf2_xchg_recv_words(32768, 13, 8, 2, 16) == 2 * 8 * 16 * w
    assert lib.cf2_xchg_send_words(32768, 13, 1, 16) == 0 and lib.cf2_xchg_recv_words(32768, 13, 8, 2, 65) == 0
    assert lib.cf2_obs_consume(None, 1, 8, 13, 1, None, None, 0, None, None, None) == -1
    assert lib.cf2_obs_rows(None, 1, 0, None, 1, 0, 1, 8, 13, None, None, None, None, 0, 8, None, None) == -1
    # depth 1 would let a pack clear its own count word: refused before any RCCL call
    h = ctypes.c_void_p()
    idb = (ctypes.c_uint8 * 128)()
    assert lib.cf2_xchg_create(idb, 128, 1, 0, 1, ctypes.byref(h)) == -1
    assert lib.cf2_xchg_create(idb, 128, 1, 0, 9, ctypes.byref(h)) == -1
    assert lib.cf2_xchg_publish(None, 0, 1, 0, None) == -1 and lib.cf2_xchg_wait(None, None) == -1
    assert lib.cf2_xchg_pred_to_host(None, None, None) == -1
    assert lib.cf2_xchg_begin(None, 1, 0, None) == -1 and lib.cf2_xchg_end(None, 0, None, None) == -1
    assert lib.cf2_xchg_step(None, None, None, None, None, None, None, None) == -1
    assert lib.cf2_xchg_run(None, None, 0, 8, 1, 0, None, 1, None, None, None, None, None, None) == -1
