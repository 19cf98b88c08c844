"""Multi-drone formations with downwash (BASELINE config 5).

The reference parses the downwash coefficients but never applies them (envs/agents.py:251-257)
and has no multi-drone env, so there is nothing of the reference to pin this to: the formula is
gym-pybullet-drones' BaseAviary._downwash (an external project, restated here from its published
code), checked below against an independent numpy restatement; the HIP kernel is checked against
the CPU restatement in tests/test_gpu_parity.py.  Parity vs PyBullet: unpinned."""
import math

import numpy as np
import pytest

import oracle as O
from cf2sim.config import ENV_SPECS, build_config

ENV = "DroneHoverBulletFreeEnvWithDownwash-v0"


def ref_downwash(p_self, others, c1=2267.18, c2=0.16, c3=-0.11, prop_radius=2.31348e-2):
    """BaseAviary._downwash: for each drone above (dz > 0) within 10 m in xy,
    alpha = c1 (r / 4 dz)^2, beta = c2 dz + c3, F += alpha exp(-0.5 (dxy / beta)^2)."""
    F = 0.0
    for q in others:
        dz = q[2] - p_self[2]
        dxy = math.hypot(q[0] - p_self[0], q[1] - p_self[1])
        if dz > 0 and dxy < 10:
            alpha = c1 * (prop_radius / (4 * dz)) ** 2
            beta = c2 * dz + c3
            F += alpha * math.exp(-0.5 * (dxy / beta) ** 2)
    return F


def test_spec_and_config():
    s = ENV_SPECS["DroneHoverBulletFreeEnvWithDownwash"]
    assert s.num_drones == 4 and s.downwash and s.registered_id == ENV
    c = build_config(ENV, 8)
    assert c.num_drones == 4 and c.downwash_on == 1
    assert tuple(c.dw_coeff) == (2267.18, 0.16, -0.11) and abs(c.prop_radius - 2.31348e-2) < 1e-12
    with pytest.raises(ValueError):
        build_config(ENV, 6)                       # whole formations only
    with pytest.raises(ValueError):
        build_config(ENV, 8, env_id_offset=2)


@pytest.mark.parametrize("seed", range(4))
def test_downwash_formula(seed):
    c = build_config(ENV, 4)
    rng = np.random.default_rng(seed)
    pos = rng.uniform([-0.3, -0.3, 0.5], [0.3, 0.3, 2.5], size=(4, 3))
    pos[1, :2] = pos[0, :2] + rng.normal(scale=0.02, size=2)      # one mate almost straight above
    for k in range(4):
        others = [pos[j] for j in range(4) if j != k]
        assert math.isclose(O.downwash(c, pos[k], pos, k), ref_downwash(pos[k], others), rel_tol=1e-12, abs_tol=1e-15)
    assert O.downwash(c, [0, 0, 1], [[0, 0, 1], [0, 0, 0.5]], 0) == 0.0      # mates below: no force


def test_formation_reset_and_downwash_effect():
    kw = dict(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0, enable_reset_distribution=False)
    env_dw = O.OracleEnv(build_config(ENV, 8, **kw), "f64")
    env_no = O.OracleEnv(build_config(ENV, 8, downwash=False, **kw), "f64")
    o = env_dw.reset()
    env_no.reset()
    sf, _ = env_dw.get_state()
    c = env_dw.cfg
    expect = np.array([[-0.25, 0, 0], [-0.25, 0, 1.0], [0.25, 0, 0], [0.25, 0, 1.0]]) + np.array(c.init_xyz)
    np.testing.assert_allclose(sf[0:3, :4].T, expect, atol=1e-12)
    np.testing.assert_allclose(sf[0:3, 4:8].T, expect, atol=1e-12)
    a = np.full((8, 4), c.hover_action, dtype=np.float32)
    env_dw.step(a)
    env_no.step(a)
    vz_dw = env_dw.get_state()[0][9]
    vz_no = env_no.get_state()[0][9]
    # lower drones (members 0, 2) are pushed down by the mate 1 m above, upper drones feel nothing
    F = ref_downwash(expect[0], [expect[1]])
    assert F > 0.05
    for k in (0, 2, 4, 6):
        assert vz_dw[k] < vz_no[k] - 1e-4
    for k in (1, 3, 5, 7):
        assert vz_dw[k] == vz_no[k]
    env_dw.close()
    env_no.close()
