"""Per-step GPU-vs-fp32-oracle error of one parity case (diagnostic, GPU box):
python tests/diag_parity_trace.py [case_index]; CF2SIM_LIB selects the library build."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as orc
from cf2sim.config import build_config
from cf2sim.vec_env import BatchedCrazyflieEnv
from test_gpu_parity import CASES, _actions
ci = int(sys.argv[1]) if len(sys.argv) > 1 else 0
env_id, kw = CASES[ci]
n, T, seed = 512, 120, 3
env = BatchedCrazyflieEnv(env_id, n, seed=seed, want_final_obs=True, **kw)
ref = orc.OracleEnv(build_config(env_id, n, seed=seed, **kw), precision="f32")
go = env.reset().cpu().numpy(); ro = ref.reset()
rng = np.random.default_rng(seed + 1)
for t in range(T):
    a = _actions(rng, n)
    g_o, g_r, g_d, g_i = env.step(torch.from_numpy(a).cuda())
    r_o, r_r, r_d, r_i = ref.step(a, want_final=True)
    g_o = g_o.cpu().numpy()
    e = np.abs(g_o - r_o) / (1 + np.abs(r_o))
    k = np.unravel_index(np.argmax(e), e.shape)
    if t % 10 == 0 or e.max() > 3e-4:
        print(f"t={t:3d} max {e.max():.2e} env {k[0]} field {k[1]} g {g_o[k]:.6f} r {r_o[k]:.6f} p99 {np.quantile(e.max(1), 0.99):.2e}", flush=True)
