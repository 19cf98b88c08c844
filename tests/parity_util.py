"""Shared helpers of the parity tests: the closed-loop test controller and the state error
metric of BASELINE.json's "state within 1e-4 rel over 240 steps"."""
import numpy as np

CLEAN = dict(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0, max_episode_steps=0)


def pd_actions(state17, hover, kp=0.5, kd=0.08, kz=0.05):
    """A stabilising attitude/altitude PD controller on obs17 = [p, q, v, w_body, a] (test helper;
    stands in for a trained policy closing the loop on the env's own observations).  kp / kd: roll
    and pitch angle / rate gains, kz: yaw-rate gain."""
    p, q, v, w = state17[:, 0:3], state17[:, 3:7], state17[:, 7:10], state17[:, 10:13]
    x, y, z, qw = q.T
    roll = np.arctan2(2 * (qw * x + y * z), 1 - 2 * (x * x + y * y))
    pitch = np.arcsin(np.clip(2 * (qw * y - z * x), -1, 1))
    T = hover + 0.5 * (1.0 - p[:, 2]) - 0.4 * v[:, 2]
    tx, ty, tz = -kp * roll - kd * w[:, 0], -kp * pitch - kd * w[:, 1], -kz * w[:, 2]
    a = (T[:, None] + tx[:, None] * np.array([-1, -1, 1, 1]) + ty[:, None] * np.array([-1, 1, 1, -1])
         + tz[:, None] * np.array([-1, 1, -1, 1]))
    return np.clip(a, -1, 1).astype(np.float32)


STATE_BLOCKS = {"pos": slice(0, 3), "quat": slice(3, 7), "vel": slice(7, 10), "omega": slice(10, 13)}


def state_rel_err(g, r):
    """Relative state error of BASELINE.json's "state within 1e-4 rel over 240 steps", per env and
    per state vector (position, quaternion, linear velocity, angular velocity):
    ||g - r||_2 / max(||r||_2, 1).  Norm-wise because a component-wise ratio is not invariant
    under a rotation of the world frame (the error of a spinning drone leaks between components);
    the floor of 1 (m, unit quaternion, m/s, rad/s) only acts on velocity vectors near hover, where
    a pure ratio is undefined.  Returns {block: [N] errors}."""
    return {k: np.linalg.norm(g[b] - r[b], axis=0) / np.maximum(np.linalg.norm(r[b], axis=0), 1.0)
            for k, b in STATE_BLOCKS.items()}
