"""The RCCL stand-in of the world-size-2 exchange tests (tests/standin_rccl; test infrastructure,
never shipped): it exports the four entry points cf2_xchg_bind resolves, its unique ids name a
shared segment both ranks open, and CF2_STANDIN_FAIL_RANK fails exactly that rank's setup.  The
all-gather itself moves device memory and runs in the -m gpu tests."""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIR = os.path.join(ROOT, "tests", "standin_rccl")
LIB = os.path.join(DIR, "_build", "libstandin_rccl.so")


def _lib():
    subprocess.run(["make", "-s", "-C", DIR], check=True)
    return ctypes.CDLL(LIB)


def test_exports_the_symbols_the_exchange_binds():
    lib = _lib()
    src = open(os.path.join(ROOT, "disturbance-crazyfile-simulation_amd", "csrc", "cf2sim_exchange.hip")).read()
    for sym in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllGather", "ncclCommDestroy"):
        assert f'dlsym(h, "{sym}")' in src
        assert hasattr(lib, sym)


def test_two_ranks_open_one_segment_and_a_failing_rank_fails_alone(monkeypatch):
    lib = _lib()

    class UniqueId(ctypes.Structure):        # ncclUniqueId, passed by value to ncclCommInitRank
        _fields_ = [("internal", ctypes.c_char * 128)]
    uid = UniqueId()
    assert lib.ncclGetUniqueId(ctypes.byref(uid)) == 0 and uid.internal.startswith(b"/cf2standin_")
    lib.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, UniqueId, ctypes.c_int]
    monkeypatch.setenv("CF2_STANDIN_SLOT_MB", "1")
    c0, c1 = ctypes.c_void_p(), ctypes.c_void_p()
    assert lib.ncclCommInitRank(ctypes.byref(c0), 2, uid, 0) == 0 and c0.value
    path = "/dev/shm" + uid.internal.decode()
    assert os.path.getsize(path) == 4096 + 2 * (1 << 20)
    monkeypatch.setenv("CF2_STANDIN_FAIL_RANK", "1")
    assert lib.ncclCommInitRank(ctypes.byref(c1), 2, uid, 1) != 0 and not c1.value
    assert lib.ncclCommInitRank(ctypes.byref(c1), 2, uid, 2) != 0          # rank out of range
    monkeypatch.setenv("CF2_STANDIN_FAIL_RANK", "-1")
    assert lib.ncclCommInitRank(ctypes.byref(c1), 2, uid, 1) == 0 and c1.value
    lib.ncclCommDestroy.argtypes = [ctypes.c_void_p]
    assert lib.ncclCommDestroy(c0) == 0 and lib.ncclCommDestroy(c1) == 0
    assert not os.path.exists(path)
