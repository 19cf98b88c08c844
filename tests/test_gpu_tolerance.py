"""Per-component tolerance report on the bench workload.

DroneHoverBulletFreeEnvWithGust-v0 with the reference-default sensor noise, 10 % domain
randomisation, motor-thrust OU noise and latency, plus Philox gusts -- bench.py's workload -- at
4096 envs for 240 env-steps, closed loop: the PD controller of tests/parity_util.py acts on each
env's own noisy observation (as a policy would), on the HIP kernel (fp32) and on the fp64
restatement (oracle/cf2_oracle.c), with the same Philox draws on both sides.  An env is compared at
every env-step before its episode ends on either side (past that point the two sides would compare
different episodes); the 240-step figures are over the envs that fly the whole window.  Two runs:
  * "gentle": gusts up to 0.4 x the HJ bound (bench: 1.5) and a softer, better damped controller
    (kp 0.3, kd 0.1), so that most drones (>= 2000 of 4096) fly all 240 steps and the step-240
    figures are over a large population;
  * "bench": the bench's 1.5 x gusts under the default controller, which crash most drones within
    the window (~430 fly all 240 steps).

For each of the 13 state components (position, quaternion x y z w, world velocity, world angular
velocity; envs/physics.py:213-250 + the restated bullet step) the table holds, over every env and
every env-step:
  max_abs   max |g - r|
  rel_p50 / rel_p99 / rel_max   |g - r| / |r| with NO floor, over samples with |r| > 1e-6
  small_frac   fraction of samples with |r| < 1e-3 (where a floor-free ratio is ill-conditioned)
  rel_rms   max_abs / rms(r) (error against the component's typical size)
and the norm-with-floor metric of the 1e-4 test (state_rel_err): ||g - r|| / max(||r||, 1) per
state vector.  The table is written to gpurun_out/tolerance_table.json (DESIGN.md section 5 quotes
it).  Parity vs PyBullet stays unpinned (the Bullet step is restated on both sides)."""
import json
import os

import numpy as np
import pytest
import torch

import oracle as O
from cf2sim.config import build_config
from parity_util import STATE_BLOCKS, pd_actions, state_rel_err

pytestmark = pytest.mark.gpu
COMP = ["px", "py", "pz", "qx", "qy", "qz", "qw", "vx", "vy", "vz", "wx", "wy", "wz"]


def _run(gust, gains, n=4096, T=240, seed=17):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env_id = "DroneHoverBulletFreeEnvWithGust-v0"
    kw = dict(max_episode_steps=0, gust_max_level=gust)
    env = BatchedCrazyflieEnv(env_id, n, seed=seed, **kw)
    cfg = build_config(env_id, n, seed=seed, **kw)
    ref = O.OracleEnv(cfg, "f64")
    sl = slice(17, 30)                     # o_k of the noisy observation: p, q, v, w
    go = env.reset().cpu().numpy()
    ro = ref.reset()
    alive = np.ones(n, bool)
    G, R, A = [], [], []
    for _ in range(T):
        go, _, gd, _ = env.step(torch.from_numpy(pd_actions(go[:, sl], cfg.hover_action, *gains)).cuda())
        go = go.cpu().numpy()
        ro, _, rd, _ = ref.step(pd_actions(ro[:, sl], cfg.hover_action, *gains))
        alive &= ~rd & ~gd.cpu().numpy().astype(bool)
        A.append(alive.copy())                 # not yet ended on either side (this step included)
        G.append(env.get_state()[0].cpu().numpy()[:13].astype(np.float64))
        R.append(ref.get_state()[0][:13].copy())
    env.close()
    ref.close()
    G, R, A = np.stack(G), np.stack(R), np.stack(A)                     # [T, 13, n], [T, n]
    table, at240 = {}, {}
    for c, name in enumerate(COMP):
        g, r = G[:, c][A], R[:, c][A]                                      # every (step, env) still flying
        err = np.abs(g - r)
        big = np.abs(r) > 1e-6
        rel = err[big] / np.abs(r[big])
        table[name] = {"max_abs": float(err.max()), "rel_p50": float(np.median(rel)),
                       "rel_p99": float(np.quantile(rel, 0.99)), "rel_max": float(rel.max()),
                       "small_frac": float(np.mean(np.abs(r) < 1e-3)),
                       "rel_rms": float(err.max() / np.sqrt(np.mean(r * r)))}
        # floor-free relative error at env-step 240 over the envs flying the whole window
        g1, r1 = G[-1, c][A[-1]], R[-1, c][A[-1]]
        e1 = np.abs(g1 - r1)
        b1 = np.abs(r1) > 1e-6
        rel1 = e1[b1] / np.abs(r1[b1])
        at240[name] = {"max_abs": float(e1.max()), "rel_p50": float(np.median(rel1)),
                       "rel_p99": float(np.quantile(rel1, 0.99)), "rel_max": float(rel1.max()),
                       "small_frac": float(np.mean(np.abs(r1) < 1e-3))}
    floor_metric = {k: float(max(state_rel_err(G[t][:, A[t]], R[t][:, A[t]])[k].max() for t in range(T)))
                    for k in STATE_BLOCKS}
    e240 = state_rel_err(G[-1][:, A[-1]], R[-1][:, A[-1]])
    final = {k: float(v.max()) for k, v in e240.items()}
    worst = np.max(np.stack(list(e240.values())), axis=0)       # per env: the worst of its four vectors
    dist240 = {"p50": float(np.median(worst)), "p99": float(np.quantile(worst, 0.99)), "max": float(worst.max()),
               "frac_within_1e-4": float(np.mean(worst < 1e-4))}
    return {"workload": f"{env_id}: gusts up to {gust} x the HJ bound + sensor noise + 10% DR + motor noise + "
                        f"latency, PD loop (kp, kd, kz = {gains}) on own obs",
            "envs": n, "env_steps": T, "env_steps_compared": int(A.sum()), "envs_flying_all_240": int(A[-1].sum()),
            "components": table, "components_at_step_240_no_floor": at240,
            "state_rel_err_max_over_steps": floor_metric, "state_rel_err_at_step_240": final,
            "state_rel_err_at_step_240_per_env": dist240}


def test_component_tolerance_table_bench_workload(gpu):
    gentle = _run(0.4, (0.3, 0.1, 0.05))
    bench = _run(1.5, (0.5, 0.08, 0.05))
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "tolerance_table.json"), "w") as f:
        json.dump({"gentle": gentle, "bench": bench, "note": "parity vs PyBullet unpinned (a7 restated on both sides)"},
                  f, indent=1)
    assert gentle["envs_flying_all_240"] >= 2000, gentle["envs_flying_all_240"]
    assert bench["envs_flying_all_240"] >= 200, bench["envs_flying_all_240"]
    # the north-star metric (floor of 1 per state vector) at env-step 240: every env of the bench
    # run; over the ~2800 envs of the gentle run, the tail of the closed loop's chaotic fp32
    # divergence reaches past 1e-4 for a few envs (their angular velocity, rad/s): held to 99 % of
    # the envs within 1e-4 and every env within 5e-4
    assert max(bench["state_rel_err_at_step_240"].values()) < 1e-4, bench["state_rel_err_at_step_240"]
    d = gentle["state_rel_err_at_step_240_per_env"]
    assert d["frac_within_1e-4"] >= 0.99 and d["max"] < 5e-4, d
    for res in (gentle, bench):
        # gross sanity: no component drifts by more than 1 % of its typical size, even in the envs
        # close to a crash (where the chaotic dynamics amplify fp32 rounding)
        assert max(v["rel_rms"] for v in res["components"].values()) < 1e-2, res["components"]
