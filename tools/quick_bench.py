import os, sys, time
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))
from cf2sim.vec_env import BatchedCrazyflieEnv
for env_id, n in [("DroneHoverBulletFreeEnvWithGust-v0", 262144), ("DroneHoverBulletFreeEnvWithRandomAdversary-v0", 65536), ("DroneHoverBulletFreeEnvWithConstWind-v0", 4096)]:
    env = BatchedCrazyflieEnv(env_id, n, seed=0)
    env.reset()
    acts = torch.rand(16, n, 4, device="cuda") * 2 - 1
    for k in range(20): env.step(acts[k % 16])
    torch.cuda.synchronize()
    K = 200
    t0 = time.perf_counter()
    for k in range(K): env.step(acts[k % 16])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / K
    print(f"{env_id} N={n}: {dt*1e6:.1f} us/step  {n/dt:.3e} env-steps/s", flush=True)
    env.close()
