"""HJ value tables as the reference stores them (distur_gener.py:155:
phoenix_drone_simulation/adversarial_generation/FasTrack_data/fastrack_{level}_15x15.npy, one file
per disturbance level, loaded with np.load): the loader finds them by the reference's file names
and path layout, and make(id, value_tables=...) steps an HJ env without touching private state."""
import os

import numpy as np
import pytest
import torch

from cf2sim.config import build_config
from cf2sim.vec_env import REFERENCE_TABLE_DIR, load_value_tables, value_table_name


def _table(seed):
    return np.random.default_rng(seed).standard_normal(15 ** 6).astype(np.float32).reshape([15] * 6)


def test_reference_file_names():
    # distur_gener.py:155 formats the level as Python prints it; Boltzmann() rounds to 1 decimal
    assert value_table_name(1.5) == "fastrack_1.5_15x15.npy"
    assert value_table_name(0.0) == "fastrack_0.0_15x15.npy"
    assert value_table_name(0.1 * 3) == "fastrack_0.3_15x15.npy"
    assert value_table_name(np.around(np.arange(0.0, 2.1, 0.1), 1)[20]) == "fastrack_2.0_15x15.npy"


@pytest.mark.parametrize("layout", ["repo_root", "table_dir"])
def test_fixed_level_env_loads_its_level_file(tmp_path, layout):
    cfg = build_config("DroneHoverBulletFreeEnvWithAdversary-v0", 4)      # level 1.5 (hover_free.py:319)
    d = tmp_path / REFERENCE_TABLE_DIR if layout == "repo_root" else tmp_path
    d.mkdir(parents=True, exist_ok=True)
    T = _table(1)
    np.save(d / "fastrack_1.5_15x15.npy", T)
    np.save(d / "fastrack_1.0_15x15.npy", _table(2))      # another level: not read
    V, tol = load_value_tables(str(tmp_path), cfg)
    assert V.shape == (1, 15 ** 6) and V.dtype == np.float32
    assert np.array_equal(V[0], T.reshape(-1))
    assert tol == [0] * int(cfg.num_levels)


def test_missing_file_and_pickled_file_are_refused(tmp_path):
    cfg = build_config("DroneHoverBulletFreeEnvWithAdversary-v0", 4)
    with pytest.raises(FileNotFoundError):
        load_value_tables(str(tmp_path), cfg)
    # an object array needs pickle: np.load(allow_pickle=False) refuses it, nothing is executed
    np.save(tmp_path / "fastrack_1.5_15x15.npy", np.array([{"a": 1}], dtype=object), allow_pickle=True)
    with pytest.raises(ValueError):
        load_value_tables(str(tmp_path), cfg)


def test_boltzmann_env_maps_each_level_to_its_table():
    cfg = build_config("DroneHoverBulletFreeEnvWithRandomHJAdversary-v0", 4)
    nl = int(cfg.num_levels)
    levels = [round(float(cfg.level_values[k]), 1) for k in range(nl)]
    a, b = _table(3), _table(4)
    V, tol = load_value_tables({lv: (a if k % 2 == 0 else b) for k, lv in enumerate(levels)}, cfg)
    assert V.shape == (2, 15 ** 6)                       # shared arrays share a row
    assert tol == [k % 2 for k in range(nl)]
    with pytest.raises(KeyError):
        load_value_tables({0.0: a}, cfg)


@pytest.mark.gpu
def test_make_steps_hj_env_from_reference_layout(gpu, tmp_path):
    """make(id, value_tables=<dir in the reference's layout>) steps without touching env._env, and
    equals binding the same table explicitly; the adapter's public bind_hj_tables does too."""
    import cf2sim
    d = tmp_path / REFERENCE_TABLE_DIR
    d.mkdir(parents=True)
    T = (np.linspace(-1, 1, 15 ** 6, dtype=np.float32) ** 3).reshape([15] * 6)
    np.save(d / "fastrack_1.5_15x15.npy", T)
    e1 = cf2sim.make("DroneHoverBulletFreeEnvWithAdversary-v0", seed=3, value_tables=str(tmp_path))
    e2 = cf2sim.make("DroneHoverBulletFreeEnvWithAdversary-v0", seed=3)
    e2.bind_hj_tables(torch.from_numpy(T.reshape(1, -1)), [0] * 21)
    o1, o2 = e1.reset(), e2.reset()
    assert np.array_equal(o1, o2)
    rng = np.random.default_rng(0)
    for _ in range(30):
        a = rng.uniform(-0.3, 0.5, 4).astype(np.float32)
        r1, r2 = e1.step(a), e2.step(a)
        assert np.array_equal(r1[0], r2[0]) and r1[1] == r2[1] and r1[2] == r2[2]
        if r1[2]:
            break
    e1.seed(3)                                           # tables stay bound across seed()
    e1.reset()
    e1.step(np.zeros(4, np.float32))
    e1.close()
    e2.close()


@pytest.mark.gpu
def test_make_info_constraint_keys(gpu):
    """compute_info's conditional keys (hover_free.py:138-166): present exactly when the matching
    constraint is violated; info['cost'] is 1 iff any is."""
    import cf2sim
    env = cf2sim.make("DroneHoverBulletFreeEnvWithoutAdversary-v0", seed=1)
    env.reset()
    seen = set()
    for t in range(200):
        a = np.full(4, 0.9 if t % 20 < 10 else -0.9, np.float32)     # tumbles, leaves the box
        if t % 7 == 3:
            a[1] = 4.0     # an unclipped policy output beyond rpy_dot_limit (deg2rad(200)): 'rpy_dot'
        _, _, done, info = env.step(a)
        keys = {"xyz_limit", "rpy", "xzy_dot", "rpy_dot"} & set(info)
        assert (info["cost"] == 1.0) == bool(keys), (t, info)
        seen |= keys
        assert "disturbance_level" in info
        if done:
            env.reset()
    assert "rpy_dot" in seen and len(seen) >= 3, seen
    env.close()
