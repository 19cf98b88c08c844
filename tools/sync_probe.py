import os, sys, time, warnings, torch
sys.path.insert(0, "disturbance-crazyfile-simulation_amd")
from cf2sim.rollout import FusedActorCritic, MLPActorCritic, collect
from cf2sim.vec_env import BatchedCrazyflieEnv
n = 262144
envs = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=0, want_final_obs=True)
ac = FusedActorCritic(MLPActorCritic().cuda(), seed=0, precision="bf16x3")
obs = envs.reset()
ro = collect(envs, ac, 32, obs=obs.clone())
ro = collect(envs, ac, 32, obs=ro.last_obs)
torch.cuda.synchronize()
torch.cuda.set_sync_debug_mode("warn")
with warnings.catch_warnings(record=True) as w:
    warnings.simplefilter("always")
    t = []
    for k in range(3):
        t0 = time.perf_counter()
        ro = collect(envs, ac, 32, obs=ro.last_obs)
        t.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    print("cpu ms per collect call", t)
    for x in w[:10]:
        print("SYNC:", str(x.message)[:200], x.filename, x.lineno)
