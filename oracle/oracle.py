"""ctypes wrapper of the CPU restatement (oracle/cf2_oracle.c).  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module,
and only as the checker / CPU baseline; the product path never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
NF, NI = 108, 5

_P = ctypes.c_void_p
_dp = ctypes.POINTER(ctypes.c_double)
_fp = ctypes.POINTER(ctypes.c_float)
_ip = ctypes.POINTER(ctypes.c_int32)
_u8p = ctypes.POINTER(ctypes.c_uint8)


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _ptr(a, t):
    return None if a is None else a.ctypes.data_as(t)


class _Lib:
    _cache: dict = {}

    @classmethod
    def get(cls, precision: str = "f64"):
        if precision not in cls._cache:
            path = os.path.join(BUILD, f"libcf2oracle_{precision}.so")
            if not os.path.exists(path):
                build()
            lib = ctypes.CDLL(path)
            lib.orc_create.restype = _P
            lib.orc_create.argtypes = [_P]
            lib.orc_destroy.argtypes = [_P]
            lib.orc_set_threads.argtypes = [_P, ctypes.c_int]
            lib.orc_set_ground_effect.argtypes = [_P, ctypes.c_int]
            lib.orc_reset.argtypes = [_P, _u8p, _dp]
            lib.orc_step.argtypes = [_P, _fp, _dp, _dp, _dp, _u8p, _u8p, _dp, _dp, _dp]
            lib.orc_physics_step.argtypes = [_P, _fp, _dp, ctypes.c_double]
            lib.orc_get_state.argtypes = [_P, _dp, _ip]
            lib.orc_set_state.argtypes = [_P, _dp, _ip]
            lib.orc_bind_tables.argtypes = [_P, _fp, ctypes.c_int, _ip]
            lib.orc_philox4x32_10.argtypes = [ctypes.POINTER(ctypes.c_uint32)] * 3
            lib.orc_t_hj.argtypes = [_P, _fp, _dp, ctypes.c_int, ctypes.c_double, _dp, _dp, _ip]
            lib.orc_t_boltzmann_index.argtypes = [_P, ctypes.c_double]
            lib.orc_t_boltzmann_index.restype = ctypes.c_int
            for name in ("orc_t_rotmat", "orc_t_quat_from_euler", "orc_t_euler_from_quat", "orc_t_quat2euler"):
                getattr(lib, name).argtypes = [_dp, _dp]
            lib.orc_t_apply_action.argtypes = [_P, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _dp]
            lib.orc_t_add_noise.argtypes = [_P] + [_dp] * 11
            lib.orc_t_bullet_substep.argtypes = [_P, _dp, _dp, _dp, _dp, ctypes.c_int, _dp]
            lib.orc_t_simple_substep.argtypes = [_P, _dp, _dp, _dp, _dp]
            lib.orc_t_reward_done_cost.argtypes = [_P, _dp, _dp, _dp, ctypes.POINTER(ctypes.c_int), _dp]
            cls._cache[precision] = lib
        return cls._cache[precision]


def downwash(cfg, pn, positions, self_index, precision="f64"):
    """orc_downwash: downwash force on drone `self_index` from the others of its group."""
    lib = _Lib.get(precision)
    fn = lib.orc_downwash
    fn.restype = ctypes.c_double if precision == "f64" else ctypes.c_float
    real = ctypes.c_double if precision == "f64" else ctypes.c_float
    M = len(positions)
    p = (real * 3)(*pn)
    arr = (real * (3 * M))(*[float(x) for row in positions for x in row])
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    return float(fn(ctypes.byref(cfg), p, arr, M, int(self_index)))


def philox(ctr, key, precision="f64"):
    lib = _Lib.get(precision)
    c = (ctypes.c_uint32 * 4)(*[int(x) & 0xFFFFFFFF for x in ctr])
    k = (ctypes.c_uint32 * 2)(*[int(x) & 0xFFFFFFFF for x in key])
    o = (ctypes.c_uint32 * 4)()
    lib.orc_philox4x32_10(c, k, o)
    return list(o)


class OracleEnv:
    """Batched env on the CPU restatement, same semantics and state layout as libcf2sim."""

    def __init__(self, cfg, precision: str = "f64"):
        self.lib = _Lib.get(precision)
        self.cfg = cfg
        self.n = int(cfg.num_envs)
        self.obs_dim = 2 * ((13 if cfg.observation_noise_on else 17) + 4)
        self.h = self.lib.orc_create(ctypes.byref(cfg))
        self._tables = None

    def close(self):
        if self.h:
            self.lib.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_threads(self, threads: int):
        """OpenMP threads of step() (formations split across threads; results are identical)."""
        self.lib.orc_set_threads(self.h, int(threads))

    def bind_tables(self, V: np.ndarray, table_of_level):
        V = np.ascontiguousarray(V, dtype=np.float32)
        t = np.ascontiguousarray(table_of_level, dtype=np.int32)
        self._tables = (V, t)
        self.lib.orc_bind_tables(self.h, _ptr(V, _fp), int(V.shape[0]), _ptr(t, _ip))

    def reset(self, mask=None):
        obs = np.zeros((self.n, self.obs_dim), np.float64)
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        self.lib.orc_reset(self.h, _ptr(m, _u8p), _ptr(obs, _dp))
        return obs

    def step(self, act, dstb=None, want_final=False):
        act = np.ascontiguousarray(act, dtype=np.float32).reshape(self.n, 4)
        d = None if dstb is None else np.ascontiguousarray(dstb, dtype=np.float64).reshape(self.n, 3)
        obs = np.zeros((self.n, self.obs_dim), np.float64)
        rew = np.zeros(self.n, np.float64)
        done = np.zeros(self.n, np.uint8)
        trunc = np.zeros(self.n, np.uint8)
        cost = np.zeros(self.n, np.float64)
        level = np.zeros(self.n, np.float64)
        fin = np.zeros((self.n, self.obs_dim), np.float64) if want_final else None
        self.lib.orc_step(self.h, _ptr(act, _fp), _ptr(d, _dp), _ptr(obs, _dp), _ptr(rew, _dp),
                          _ptr(done, _u8p), _ptr(trunc, _u8p), _ptr(cost, _dp), _ptr(level, _dp),
                          _ptr(fin, _dp))
        info = dict(cost=cost, truncated=trunc.astype(bool), level=level)
        if want_final:
            info["final_obs"] = fin
        return obs, rew, done.astype(bool), info

    def set_ground_effect(self, on: bool):
        """BasePhysics.use_ground_effect of this context (orc_set_ground_effect)."""
        self.lib.orc_set_ground_effect(self.h, int(bool(on)))

    def physics_step(self, act, dstb=None, time_step=0.0):
        """One physics sub-step of every env (orc_physics_step; the plugin's step_forward)."""
        act = np.ascontiguousarray(act, dtype=np.float32).reshape(self.n, 4)
        d = None if dstb is None else np.ascontiguousarray(dstb, dtype=np.float64).reshape(self.n, 3)
        self.lib.orc_physics_step(self.h, _ptr(act, _fp), _ptr(d, _dp), float(time_step))

    def get_state(self):
        sf = np.zeros((NF, self.n), np.float64)
        si = np.zeros((NI, self.n), np.int32)
        self.lib.orc_get_state(self.h, _ptr(sf, _dp), _ptr(si, _ip))
        return sf, si

    def set_state(self, sf, si):
        sf = np.ascontiguousarray(sf, dtype=np.float64)
        si = np.ascontiguousarray(si, dtype=np.int32)
        self.lib.orc_set_state(self.h, _ptr(sf, _dp), _ptr(si, _ip))


# ---- component functions (golden-vector tests) ----
def _vec(fn, x, n_out, precision="f64"):
    lib = _Lib.get(precision)
    x = np.ascontiguousarray(x, dtype=np.float64)
    o = np.zeros(n_out, np.float64)
    getattr(lib, fn)(_ptr(x, _dp), _ptr(o, _dp))
    return o


def rotmat(q, precision="f64"):
    return _vec("orc_t_rotmat", q, 9, precision).reshape(3, 3)


def quat_from_euler(e, precision="f64"):
    return _vec("orc_t_quat_from_euler", e, 4, precision)


def euler_from_quat(q, precision="f64"):
    return _vec("orc_t_euler_from_quat", q, 3, precision)


def quat2euler(q, precision="f64"):
    return _vec("orc_t_quat2euler", q, 3, precision)


def hj(cfg, V, states, level, precision="f64"):
    lib = _Lib.get(precision)
    V = np.ascontiguousarray(V, dtype=np.float32)
    s = np.ascontiguousarray(states, dtype=np.float64).reshape(-1, 6)
    n = s.shape[0]
    d = np.zeros((n, 3)); u = np.zeros((n, 3)); idx = np.zeros((n, 6), np.int32)
    lib.orc_t_hj(ctypes.byref(cfg), _ptr(V, _fp), _ptr(s, _dp), n, float(level), _ptr(d, _dp), _ptr(u, _dp),
                 _ptr(idx, _ip))
    return d, u, idx


def boltzmann_index(cfg, u, precision="f64"):
    return _Lib.get(precision).orc_t_boltzmann_index(ctypes.byref(cfg), float(u))


def apply_action(cfg, acts, ou_normals, init_x, init_buf, precision="f64"):
    lib = _Lib.get(precision)
    acts = np.ascontiguousarray(acts, np.float64).reshape(-1, 4)
    T = acts.shape[0]
    n = np.ascontiguousarray(ou_normals, np.float64).reshape(T, 4)
    x0 = np.ascontiguousarray(init_x, np.float64)
    b0 = np.ascontiguousarray(init_buf, np.float64).reshape(-1)
    f = np.zeros((T, 4)); tz = np.zeros(T); xs = np.zeros((T, 4))
    lib.orc_t_apply_action(ctypes.byref(cfg), T, _ptr(acts, _dp), _ptr(n, _dp), _ptr(x0, _dp), _ptr(b0, _dp),
                           _ptr(f, _dp), _ptr(tz, _dp), _ptr(xs, _dp))
    return f, tz, xs


def add_noise(cfg, pos, vel, rot, omega, normals, uniforms, bias, precision="f64"):
    lib = _Lib.get(precision)
    arr = [np.ascontiguousarray(a, np.float64) for a in (pos, vel, rot, omega, normals, uniforms)]
    b = np.array(bias, np.float64)
    op, ov, orr, oo = (np.zeros(3) for _ in range(4))
    lib.orc_t_add_noise(ctypes.byref(cfg), *[_ptr(a, _dp) for a in arr], _ptr(b, _dp), _ptr(op, _dp),
                        _ptr(ov, _dp), _ptr(orr, _dp), _ptr(oo, _dp))
    return op, ov, orr, oo, b


def bullet_substep(cfg, st, a, dstb, ou_n, first_after_reset=False, precision="f64"):
    lib = _Lib.get(precision)
    s = np.array(st, np.float64)
    out = np.zeros(6)
    lib.orc_t_bullet_substep(ctypes.byref(cfg), _ptr(s, _dp), _ptr(np.asarray(a, np.float64), _dp),
                             _ptr(np.asarray(dstb, np.float64), _dp), _ptr(np.asarray(ou_n, np.float64), _dp),
                             int(first_after_reset), _ptr(out, _dp))
    return s, out


def simple_substep(cfg, st, a, ou_n, ou, precision="f64"):
    lib = _Lib.get(precision)
    s = np.array(st, np.float64)
    o = np.array(ou, np.float64)
    lib.orc_t_simple_substep(ctypes.byref(cfg), _ptr(s, _dp), _ptr(np.asarray(a, np.float64), _dp),
                             _ptr(np.asarray(ou_n, np.float64), _dp), _ptr(o, _dp))
    return s, o


def reward_done_cost(cfg, attrs, a, precision="f64"):
    lib = _Lib.get(precision)
    r = ctypes.c_double(); d = ctypes.c_int(); c = ctypes.c_double()
    lib.orc_t_reward_done_cost(ctypes.byref(cfg), _ptr(np.asarray(attrs, np.float64), _dp),
                               _ptr(np.asarray(a, np.float64), _dp), ctypes.byref(r), ctypes.byref(d),
                               ctypes.byref(c))
    return r.value, bool(d.value), c.value
