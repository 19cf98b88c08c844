"""ctypes binding of libcf2sim.so (the C ABI declared in include/cf2sim.h).

The shared library is built in-tree by ``cf2sim.build.build_native()`` (hipcc, gfx950) and
loaded here.  There is no fallback: if the library or a GPU is missing, every entry point
raises.  torch must be imported first so that the HIP runtime torch ships
(soname libamdhip64.so.7) is the one libcf2sim binds to, and device pointers / streams
handed over from torch are valid in it.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (loads the process' HIP runtime before libcf2sim)

from .config import CF2Config

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CF2SIM_LIB") or os.path.join(PKG_DIR, "libcf2sim.so")   # override: A/B builds
REPO_INCLUDE = os.path.abspath(os.path.join(PKG_DIR, "..", "..", "include", "cf2sim.h"))

# every symbol include/cf2sim.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    "cf2_abi_version", "cf2_config_sizeof", "cf2_status_string", "cf2_last_hip_error", "cf2_device_errors",
    "cf2_create", "cf2_destroy", "cf2_layout_get", "cf2_bind_hj_tables", "cf2_reset", "cf2_step", "cf2_collect_step",
    "cf2_collect_rollout", "cf2_physics_step",
    "cf2_set_ground_effect",
    "cf2_rollout", "cf2_get_state", "cf2_set_state", "cf2_hj_disturbance",
    "cf2_policy_weights_count", "cf2_policy_packed_count", "cf2_policy_pack", "cf2_policy_forward", "cf2_value_forward_masked", "cf2_gae",
    "cf2_hbm_probe", "cf2_step_packed", "cf2_obs_packed_words", "cf2_xchg_send_words", "cf2_obs_pack", "cf2_obs_consume", "cf2_obs_rows",
    "cf2_xchg_bind", "cf2_xchg_unique_id", "cf2_xchg_create", "cf2_xchg_destroy", "cf2_xchg_register",
    "cf2_xchg_publish", "cf2_xchg_wait_free", "cf2_xchg_wait", "cf2_xchg_pred_to_host", "cf2_xchg_begin", "cf2_xchg_step", "cf2_xchg_end", "cf2_xchg_env_step", "cf2_xchg_run",
    "cf2_xchg_host_times", "cf2_xchg_copy_sync",
    "cf2_xchg_recv_words",
)


class CF2Layout(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "num_envs", "num_float_fields", "num_int_fields", "obs_dim", "obs_len",
        "f_pos", "f_quat", "f_vel", "f_omega", "f_rpy", "f_motor", "f_ou", "f_abuf", "f_bias", "f_lpf", "f_held",
        "f_obs_prev", "f_hist_act", "f_param", "f_dstb", "i_ep_step", "i_rng", "i_flags", "i_level", "i_gust",
        "num_params", "f_motor_lo")]


CF2_ERR_UNSUPPORTED = -4      # include/cf2sim.h cf2_status


class CF2Error(RuntimeError):
    pass


_lib = None


def load() -> ctypes.CDLL:
    """Load libcf2sim.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CF2Error(f"{LIB_PATH} not found: run `python -c 'import __graft_entry__ as g; g.build()'` "
                       "(hipcc --offload-arch=gfx950) first")
    lib = ctypes.CDLL(LIB_PATH)
    P, vp = ctypes.POINTER, ctypes.c_void_p
    lib.cf2_abi_version.restype = ctypes.c_int
    lib.cf2_config_sizeof.restype = ctypes.c_size_t
    lib.cf2_policy_weights_count.restype = ctypes.c_size_t
    lib.cf2_policy_packed_count.restype = ctypes.c_size_t
    lib.cf2_status_string.restype = ctypes.c_char_p
    lib.cf2_status_string.argtypes = [ctypes.c_int]
    lib.cf2_last_hip_error.restype = ctypes.c_int
    lib.cf2_create.argtypes = [P(CF2Config), P(vp)]
    lib.cf2_destroy.argtypes = [vp]
    lib.cf2_device_errors.argtypes = [vp, P(ctypes.c_uint32), ctypes.c_int]
    lib.cf2_layout_get.argtypes = [vp, P(CF2Layout)]
    lib.cf2_bind_hj_tables.argtypes = [vp, vp, ctypes.c_int, P(ctypes.c_int32)]
    lib.cf2_reset.argtypes = [vp, vp, vp, vp]
    lib.cf2_step.argtypes = [vp] * 11
    lib.cf2_physics_step.argtypes = [vp, vp, vp, ctypes.c_float, vp]
    lib.cf2_collect_step.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_int, ctypes.c_uint64,
                                     ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp, vp]
    lib.cf2_collect_rollout.argtypes = [vp, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_int,
                                        ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp]
    lib.cf2_set_ground_effect.argtypes = [vp, ctypes.c_int]
    lib.cf2_rollout.argtypes = [vp, ctypes.c_int, vp, ctypes.c_size_t, vp, vp, vp, vp, vp, vp, vp, vp]
    lib.cf2_get_state.argtypes = [vp, vp, vp, vp]
    lib.cf2_set_state.argtypes = [vp, vp, vp, vp]
    lib.cf2_hj_disturbance.argtypes = [P(CF2Config), vp, vp, ctypes.c_uint32, ctypes.c_float, vp, vp, vp]
    u32 = ctypes.c_uint32
    lib.cf2_policy_weights_count.argtypes = [u32]
    lib.cf2_policy_packed_count.argtypes = [u32, ctypes.c_int]
    lib.cf2_policy_pack.argtypes = [vp, u32, ctypes.c_int, vp, vp]
    lib.cf2_policy_forward.argtypes = [vp, u32, u32, ctypes.c_int, vp, ctypes.c_uint64, u32, u32, ctypes.c_int, vp, vp,
                                       vp, vp]
    lib.cf2_value_forward_masked.argtypes = [vp, u32, u32, ctypes.c_int, vp, vp, vp, vp]
    lib.cf2_gae.argtypes = [u32, u32, vp, vp, vp, vp, vp, vp, ctypes.c_float, ctypes.c_float, ctypes.c_float, vp, vp,
                            vp, vp]
    lib.cf2_hbm_probe.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, vp]
    lib.cf2_obs_packed_words.restype = ctypes.c_size_t
    lib.cf2_obs_packed_words.argtypes = [u32, u32, u32]
    lib.cf2_obs_pack.argtypes = [vp, vp, u32, u32, u32, vp, vp, vp, vp]
    lib.cf2_step_packed.argtypes = [vp] * 10 + [u32, vp]
    lib.cf2_xchg_send_words.restype = ctypes.c_size_t
    lib.cf2_xchg_send_words.argtypes = [u32, u32, u32, u32]
    lib.cf2_xchg_recv_words.restype = ctypes.c_size_t
    lib.cf2_xchg_recv_words.argtypes = [u32, u32, u32, u32, u32]
    lib.cf2_obs_consume.argtypes = [vp, u32, u32, u32, u32, vp, vp, u32, vp, vp, vp]
    lib.cf2_obs_rows.argtypes = [vp, u32, u32, vp, u32, u32, u32, u32, u32, vp, vp, vp, vp, u32, u32, vp, vp]
    lib.cf2_xchg_bind.argtypes = [ctypes.c_char_p]
    lib.cf2_xchg_unique_id.argtypes = [vp, ctypes.c_size_t]
    lib.cf2_xchg_create.argtypes = [vp, ctypes.c_size_t, u32, u32, u32, P(vp)]
    lib.cf2_xchg_destroy.argtypes = [vp]
    lib.cf2_xchg_register.argtypes = [vp, u32, u32, u32, u32, vp, vp, vp, vp, vp, vp, vp, u32]
    lib.cf2_xchg_publish.argtypes = [vp, ctypes.c_uint64, u32, u32, vp]
    lib.cf2_xchg_wait_free.argtypes = [vp, u32, vp]
    lib.cf2_xchg_wait.argtypes = [vp, vp]
    lib.cf2_xchg_pred_to_host.argtypes = [vp, vp, vp]
    lib.cf2_xchg_begin.argtypes = [vp, u32, u32, vp]
    lib.cf2_xchg_step.argtypes = [vp] * 8
    lib.cf2_xchg_end.argtypes = [vp, ctypes.c_uint64, vp, vp]
    lib.cf2_xchg_env_step.argtypes = [vp, vp, ctypes.c_uint64, u32, u32, vp, vp, vp, vp, vp, vp, vp]
    lib.cf2_xchg_run.argtypes = [vp, vp, ctypes.c_uint64, u32, u32, u32, vp, u32, vp, vp, vp, vp, vp, vp]
    lib.cf2_xchg_host_times.argtypes = [vp, vp, u32, vp, ctypes.c_int]
    lib.cf2_xchg_copy_sync.argtypes = [vp, vp]
    for name in EXPORTED_SYMBOLS:
        if name not in ("cf2_abi_version", "cf2_config_sizeof", "cf2_status_string", "cf2_last_hip_error",
                        "cf2_policy_weights_count", "cf2_policy_packed_count", "cf2_obs_packed_words",
                        "cf2_xchg_send_words", "cf2_xchg_recv_words"):
            getattr(lib, name).restype = ctypes.c_int
    if lib.cf2_config_sizeof() != ctypes.sizeof(CF2Config):
        raise CF2Error(f"cf2_config size mismatch: C {lib.cf2_config_sizeof()} vs Python {ctypes.sizeof(CF2Config)}")
    _lib = lib
    return lib


def check(status: int, what: str = "cf2 call"):
    if status != 0:
        lib = load()
        msg = lib.cf2_status_string(status).decode()
        raise CF2Error(f"{what} failed: {msg} (status {status}, hip error {lib.cf2_last_hip_error()})")


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None passes NULL)."""
    return None if t is None else t.data_ptr()
