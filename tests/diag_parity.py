"""Print GPU-vs-oracle divergence per env id over T env-steps (diagnostic, GPU box; kept under
tests/ because it runs the oracle: python tests/diag_parity.py)."""
import os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as orc
from cf2sim.config import build_config
from cf2sim.vec_env import BatchedCrazyflieEnv

CASES = [
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", {}),
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", dict(observation_noise=0, domain_randomization=-1, motor_thrust_noise=0)),
    ("DroneHoverSimpleEnv-v0", {}),
    ("DroneHoverBulletEnvWithRandomAdversary-v0", {}),
    ("DroneHoverBulletFreeEnvWithGust-v0", {}),
    ("DroneHoverBulletFreeEnvWithConstWind-v0", {}),
    ("DroneHoverBulletEnv-v0", dict(observation_noise=0)),
]
T = int(os.environ.get("T", "240")); n = int(os.environ.get("N", "512"))
for env_id, kw in CASES:
    for prec in ("f32", "f64"):
        env = BatchedCrazyflieEnv(env_id, n, seed=3, **kw)
        ref = orc.OracleEnv(build_config(env_id, n, seed=3, **kw), precision=prec)
        o = env.reset().cpu().numpy(); ro = ref.reset()
        e0 = np.abs(o - ro).max()
        rng = np.random.default_rng(1)
        worst = []; dmis = 0
        for t in range(T):
            a = (rng.uniform(-1, 1, size=(n, 4)) * 0.2 + 0.1111).astype(np.float32)
            go, gr, gd, gi = env.step(torch.from_numpy(a).cuda())
            ro, rr, rd, ri = ref.step(a)
            go = go.cpu().numpy(); gd = gd.cpu().numpy().astype(bool)
            dmis += int((gd != rd).sum())
            err = np.abs(go - ro); rel = err / (np.abs(ro) + 1e-3)
            worst.append((err.max(), np.quantile(err.max(1), 0.99), np.abs(gr.cpu().numpy() - rr).max()))
        sf, si = env.get_state(); rsf, rsi = ref.get_state()
        serr = np.abs(sf.cpu().numpy()[:13] - rsf[:13]).max()
        w = np.array(worst)
        print(f"{env_id:48s} {str(kw)[:40]:40s} {prec}: reset {e0:.2e} | obs max@10 {w[:10,0].max():.2e} @60 {w[:60,0].max():.2e} @{T} {w[:,0].max():.2e} p99 {w[:,1].max():.2e} | rew {w[:,2].max():.2e} | done mismatches {dmis} | state13 {serr:.2e} | ep_step eq {(si.cpu().numpy()[0]==rsi[0]).mean():.3f}", flush=True)
        env.close()
