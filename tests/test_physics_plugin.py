"""The physics-plugin contract: the reference builds its physics by
name around the env's drone (envs/base.py:223-232) and drives it with step_forward(action[, dstb])
and set_parameters(time_step, number_solver_iterations) (envs/physics.py:8-76, 79-124, 127-200,
202-250).  cf2sim.physics mirrors that contract over the HIP physics kernel (cf2_physics_step);
the GPU tests step it through the reference's getattr lookup against the CPU restatement's
orc_physics_step (same sub-step, same Philox OU draws)."""
import inspect

import numpy as np
import pytest

import oracle as O
from cf2sim.config import build_config

NAMES = ["PyBulletPhysics", "PybulletPhysicsWithAdversary", "SimplePhysics", "HipBatchedPhysics"]


def test_plugin_classes_resolve_by_name_with_reference_signatures():
    import cf2sim.physics as phoenix_physics
    for name in NAMES:
        assert hasattr(phoenix_physics, name)                     # base.py:224-225
        cls = getattr(phoenix_physics, name)                      # base.py:226
        params = list(inspect.signature(cls.__init__).parameters)
        assert params[:4] == ["self", "drone", "bc", "time_step"]  # physics.py:11-19
        assert {"gravity", "number_solver_iterations", "use_ground_effect"} <= set(params)
        assert list(inspect.signature(cls.set_parameters).parameters)[:3] == ["self", "time_step",
                                                                            "number_solver_iterations"]
        assert callable(cls.step_forward)
    with pytest.raises(AssertionError, match="not found"):
        phoenix_physics.resolve_physics("MuJoCoPhysics", 0)
    with pytest.raises(TypeError):
        phoenix_physics.PyBulletPhysics(object(), None, time_step=0.005)


def _pair(env_id, n, seed, kw):
    from cf2sim.physics import BatchedDrone
    drone = BatchedDrone(num_drones=n, seed=seed, env_id=env_id, **kw)
    ref = O.OracleEnv(build_config(env_id, n, seed=seed, auto_reset=False, max_episode_steps=0, **kw), "f32")
    return drone, ref


def _err(g, r):
    return float((np.abs(g - r) / (1.0 + np.abs(r))).max())


@pytest.mark.gpu
@pytest.mark.parametrize("name,env_id,kw,time_step", [
    ("PybulletPhysicsWithAdversary", "DroneHoverBulletFreeEnvWithoutAdversary-v0", {}, None),
    ("PyBulletPhysics", "DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(domain_randomization=-1), 0.005),
    ("SimplePhysics", "DroneHoverSimpleEnv-v0", {}, None),
    ("HipBatchedPhysics", "DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(latency=0.0), 0.004),
    ("PybulletPhysicsWithAdversary+ground_effect", "DroneHoverBulletFreeEnvWithoutAdversary-v0", {}, None),
])
def test_plugin_step_forward_matches_restatement(gpu, name, env_id, kw, time_step):
    """getattr(cf2sim.physics, name)(drone, bc, time_step=...) stepped 60 sub-steps with random
    actions (and adversary torques where the class takes them) vs the fp32 restatement: state
    within 2e-5 mixed abs/rel (the fused-FMA / approximate-transcendental differences of the
    kernel), counters exact."""
    import torch
    import cf2sim.physics as phoenix_physics
    n, seed = 256, 5
    name, _, ge = name.partition("+")
    drone, ref = _pair(env_id, n, seed, kw)
    phys = getattr(phoenix_physics, name)(drone, None, time_step=time_step, use_ground_effect=bool(ge))
    phys.set_parameters(time_step=time_step, number_solver_iterations=5)
    drone.reset()
    ref.reset()
    if ge:
        # the batch starts 3-30 cm above the ground.  Lower is ill-conditioned in any precision:
        # GND_EFF_H_CLIP is 3.7 um (agents.py:156), so (r/4z)^2 grows without practical bound as a
        # prop nears z = 0 (x2.8e7 thrust at the clip), where PyBullet's ground plane would be hit
        ref.set_ground_effect(True)
        gsf, gsi = drone.env.get_state()
        z = np.random.default_rng(2).uniform(0.03, 0.3, n)
        gsf[2] = torch.from_numpy(z.astype(np.float32))
        drone.env.set_state(gsf, gsi)
        rsf, rsi = ref.get_state()
        rsf[2] = z.astype(np.float32)
        ref.set_state(rsf, rsi)
    rng = np.random.default_rng(1)
    takes_dstb = name in ("PybulletPhysicsWithAdversary", "HipBatchedPhysics")
    zmin = np.full(n, np.inf)
    for _ in range(60):
        a = (rng.uniform(-1, 1, (n, 4)) * 0.3 + 0.1111).astype(np.float32)
        d = (rng.uniform(-1, 1, (n, 3)) * 2e-4).astype(np.float32) if takes_dstb else None
        at = torch.from_numpy(a).cuda()
        if takes_dstb:
            phys.step_forward(at, torch.from_numpy(d).cuda())
        else:
            phys.step_forward(at)
        ref.physics_step(a, d, time_step or 0.0)
        if ge:
            zmin = np.minimum(zmin, ref.get_state()[0][2])
    gsf, gsi = drone.env.get_state()
    rsf, rsi = ref.get_state()
    gsf, gsi = gsf.cpu().numpy(), gsi.cpu().numpy()
    L = drone.env.layout
    fields = list(range(0, 13)) + list(range(L.f_motor, L.f_motor + 8))
    # with ground effect only the drones that stayed >= 5 cm up are compared: below that fp32
    # and fp64 restatements themselves part by >2e-4 within 60 sub-steps (the 1/z^2 thrust)
    keep = zmin >= 0.05
    assert keep.sum() >= n // 3
    assert _err(gsf[fields][:, keep], rsf[fields][:, keep]) < 2e-5
    np.testing.assert_array_equal(gsi[:3], rsi[:3])        # episode step, RNG counter, flags
    # the agent attributes read back from the snapshot
    np.testing.assert_allclose(drone.xyz.cpu().numpy()[keep], rsf[0:3].T[keep], rtol=0, atol=2e-5)
    np.testing.assert_allclose(drone.quaternion.cpu().numpy()[keep], rsf[3:7].T[keep], rtol=0, atol=2e-5)
    if name != "SimplePhysics":
        rpy = drone.rpy.cpu().numpy()[keep]
        q = rsf[3:7].T[keep]
        x, y, z, w = q.T
        roll = np.arctan2(2 * (y * z + w * x), w * w - x * x - y * y + z * z)
        np.testing.assert_allclose(rpy[:, 0], roll, atol=1e-4)
    drone.close()
    ref.close()


@pytest.mark.gpu
def test_plugin_rejects_mismatched_drone_and_bad_inputs(gpu):
    import torch
    import cf2sim.physics as phoenix_physics
    drone = phoenix_physics.BatchedDrone("cf21x_bullet", num_drones=8)
    with pytest.raises(ValueError):
        phoenix_physics.SimplePhysics(drone, None, time_step=0.005)
    phys = phoenix_physics.PybulletPhysicsWithAdversary(drone, None, time_step=0.005)
    with pytest.raises(ValueError):
        phys.step_forward(torch.zeros(8, 3, device="cuda"), torch.zeros(8, 3, device="cuda"))
    with pytest.raises(ValueError):
        phys.step_forward(torch.zeros(8, 4, device="cuda"), torch.zeros(8, device="cuda"))
    simple = phoenix_physics.BatchedDrone("cf21x_sys_eq", num_drones=8)
    with pytest.raises(ValueError):            # SimplePhysics has no ground effect (physics.py:127-200)
        phoenix_physics.SimplePhysics(simple, None, time_step=0.005, use_ground_effect=True)
    phoenix_physics.PyBulletPhysics(drone, None, time_step=0.005, use_ground_effect=True)
    from cf2sim._native import CF2Error
    with pytest.raises(CF2Error, match="unsupported|UNSUPPORTED|outside"):   # env-steps carry no ground effect
        drone.env.step(torch.zeros(8, 4, device="cuda"))
    simple.close()
    drone.close()


@pytest.mark.gpu
def test_prop_spin_up_reaction_is_the_rotors_angular_momentum(gpu):
    """Known answer for the prop joints' spin dynamics in the Bullet sub-step (a7: bullet3's
    btMultiBody behind bc.stepSimulation(), envs/physics.py:249; the reference spins the prop joints
    with setJointMotorControl2(targetVelocity = x_i * 100), envs/agents.py:323-328).  Vs PyBullet this
    stays unpinned; this checks the kernel against angular-momentum conservation instead of against
    the builder's own restatement.

    From rest (identity attitude, zero velocity and body rates, all four motors in the same state,
    the props already spinning), one cf2_physics_step whose action changes the motor targets
    unevenly.  About the yaw axis the body and its four rotors (inertia Ip each, joint axes
    a = (-1, +1, -1, +1), joint speeds w_j = prop_speed_gain * x_j) hold
        L_z = (Izz + 4 Ip) wz + Ip * sum_j a_j w_j,
    which changes only by the external yaw-torque impulse tau dt (the mixer's yaw torque: the same
    in a run with Ip = 0, whose rotors carry no momentum).  With the prop mass set to 0 (so the
    locked props add only Ip to the composite inertia) and no damping torque at zero rates:
        (Izz + 4 Ip) wz(Ip) = Izz wz(0) - Ip * sum_j a_j (w_j' - w_j).
    The gyroscopic coupling w x L is zero at zero body rates; the motor states after the sub-step
    (w_j') are read back from the kernel."""
    import torch
    import cf2sim.physics as phoenix_physics
    from cf2sim.physics import BatchedDrone
    n = 64
    env_id = "DroneHoverBulletFreeEnvWithoutAdversary-v0"
    rng = np.random.default_rng(4)
    a = np.full((n, 4), 0.1, np.float32)
    # motor 0's target differs from the other three's (0.1) by 0.4-1.0, per drone
    a[:, 0] = (rng.choice([-1.0, 1.0], n) * rng.uniform(0.5, 0.9, n)).astype(np.float32)
    res = {}
    for ip in ("urdf", 0.0):
        cfg = build_config(env_id, n, seed=1, auto_reset=False, max_episode_steps=0, latency=0.0,
                           motor_thrust_noise=0.0, observation_noise=0, domain_randomization=-1)
        ip_val = float(cfg.prop_inertia) if ip == "urdf" else 0.0
        cfg.prop_inertia = ip_val
        cfg.prop_mass = 0.0
        drone = BatchedDrone(config=cfg, env_id=env_id)
        phys = phoenix_physics.PyBulletPhysics(drone, None, time_step=None)
        drone.reset()
        env, L = drone.env, drone.env.layout
        sf, si = env.get_state()
        sf[L.f_pos:L.f_pos + 3] = torch.tensor([0.0, 0.0, 1.0], device=sf.device)[:, None]
        sf[L.f_quat:L.f_quat + 4] = torch.tensor([0.0, 0.0, 0.0, 1.0], device=sf.device)[:, None]
        sf[L.f_vel:L.f_vel + 3] = 0.0
        sf[L.f_omega:L.f_omega + 3] = 0.0
        sf[L.f_motor:L.f_motor + 4] = 0.5
        sf[L.f_motor_lo:L.f_motor_lo + 4] = 0.0
        sf[L.f_ou:L.f_ou + 4] = 0.0
        si[L.i_flags] |= 1 << 7                      # a sub-step ran since the reset: the props spin
        env.set_state(sf, si)
        x_prev = env.get_state()[0][L.f_motor:L.f_motor + 4].cpu().numpy().astype(np.float64)
        phys.step_forward(torch.from_numpy(a).cuda())
        sf2, _ = env.get_state()
        x_new = sf2[L.f_motor:L.f_motor + 4].cpu().numpy().astype(np.float64)
        wz = sf2[L.f_omega + 2].cpu().numpy().astype(np.float64)
        izz = float(np.float32(cfg.izz))
        kq = float(np.float32(cfg.prop_speed_gain))
        res[ip] = (wz, x_prev, x_new, izz, kq, float(np.float32(ip_val)))
        env.check_device_errors()
        drone.close()
    wz_a, xp, xn, izz, kq, ip = res["urdf"]
    wz_b, xp_b, xn_b, _, _, _ = res[0.0]
    assert ip > 0 and kq > 0
    np.testing.assert_array_equal(xn, xn_b)          # the same motor states: the same thrusts and yaw torque
    ax = np.array([-1.0, 1.0, -1.0, 1.0])
    dsp = kq * ((xn - xp) * ax[:, None]).sum(0)     # change of sum_j a_j w_j
    assert np.abs(dsp).min() > 0.5                   # the rotors' momentum changes in every drone
    lhs = (izz + 4 * ip) * wz_a
    rhs = izz * wz_b - ip * dsp
    reaction = ip * np.abs(dsp)
    assert np.all(np.abs(lhs - rhs) <= 2e-3 * reaction), (np.abs(lhs - rhs) / reaction).max()
    # and the reaction is a visible share of the yaw-rate response
    assert np.all(np.abs(wz_a - wz_b) > 1e-2 * reaction / izz)
