import sys, torch
sys.path.insert(0, "disturbance-crazyfile-simulation_amd")
from cf2sim.vec_env import BatchedCrazyflieEnv
env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", 262144, seed=0)
env.reset()
acts = torch.rand(8, 262144, 4, device=env.device) * 2 - 1
tot = 0
for k in range(300):
    o, r, d, info = env.step(acts[k % 8])
    if k >= 100: tot += d.float().mean().item()
print("done rate per env-step", tot / 200)
