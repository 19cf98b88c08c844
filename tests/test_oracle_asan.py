"""The CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer:
`make -C oracle asan` builds oracle/asan_driver.c against cf2_oracle.c (fp64 and fp32 builds) and
this test runs it on the config of every registered hover env and the extension configs (HJ
tables, formations, external disturbance, latency / aggregation variants).  Any sanitizer report
aborts the driver (-fno-sanitize-recover=all)."""
import ctypes
import fcntl
import os
import subprocess

import pytest

from cf2sim.config import build_config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CASES = [
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", {}),
    ("DroneHoverBulletFreeEnvWithGust-v0", {}),
    ("DroneHoverBulletFreeEnvWithConstWind-v0", {}),
    ("DroneHoverBulletEnvWithRandomAdversary-v0", {}),
    ("DroneHoverSimpleEnv-v0", {}),
    ("DroneHoverBulletFreeEnvWithRandomHJAdversary-v0", {}),
    ("DroneHoverBulletFreeEnvWithDownwash-v0", {}),
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(aggregate_phy_steps=1, latency=0.02)),
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(observation_noise=0, domain_randomization=-1,
                                                         latency=0.0, max_episode_steps=20)),
]


@pytest.fixture(scope="module")
def drivers():
    # pytest-xdist workers each build the fixture: serialise make so no worker runs a half-linked driver
    os.makedirs(os.path.join(ROOT, "oracle", "_build"), exist_ok=True)
    with open(os.path.join(ROOT, "oracle", "_build", ".asan.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail("make asan failed:\n" + r.stderr[-2000:])
    return [os.path.join(ROOT, "oracle", "_build", f"asan_driver_{p}") for p in ("f64", "f32")]


@pytest.mark.parametrize("env_id,kw", CASES)
def test_restatement_is_sanitizer_clean(drivers, tmp_path, env_id, kw):
    cfg = build_config(env_id, 24, seed=3, **kw)
    blob = tmp_path / "cfg.bin"
    blob.write_bytes(ctypes.string_at(ctypes.addressof(cfg), ctypes.sizeof(cfg)))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    for exe in drivers:
        r = subprocess.run([exe, str(blob), "60"], capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0 and r.stdout.startswith("ok"), (exe, r.stdout[-500:], r.stderr[-3000:])
        assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-3000:]
