"""Probe: does a collect split into S row shards, each on its own HIP stream, overlap one shard's
policy forward with another's env-step?  Per step every shard runs policy -> env on its stream
(the shards are independent, so the streams never wait on each other).
python tools/overlap_probe.py [--envs N] [--shards 1 2 4] [--steps T] [--prio]"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=262144)
    ap.add_argument("--shards", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    ap.add_argument("--prio", action="store_true", help="policy streams at high priority")
    args = ap.parse_args()
    from cf2sim import _native
    from cf2sim.rollout import FusedActorCritic, MLPActorCritic
    from cf2sim.vec_env import BatchedCrazyflieEnv
    lib = _native.load()
    ac = MLPActorCritic(obs_dim=34).cuda()
    fused = FusedActorCritic(ac, seed=0)
    out = []
    for S in args.shards:
        m = args.envs // S
        envs = [BatchedCrazyflieEnv(args.env_id, m, seed=1, env_id_offset=s * m, want_final_obs=True) for s in range(S)]
        d = envs[0].obs_dim
        T = args.steps
        obs = torch.empty(T + 1, args.envs, d, device="cuda")
        act = torch.empty(T, args.envs, 4, device="cuda")
        val = torch.empty(T, args.envs, device="cuda")
        lp = torch.empty(T, args.envs, device="cuda")
        rew = torch.empty(T, args.envs, device="cuda")
        d8 = torch.empty(T, args.envs, dtype=torch.uint8, device="cuda")
        t8 = torch.empty(T, args.envs, dtype=torch.uint8, device="cuda")
        fin = torch.empty(T, args.envs, d, device="cuda")
        for s, e in enumerate(envs):
            obs[0, s * m:(s + 1) * m] = e.reset()
        streams = [torch.cuda.Stream(priority=-1 if args.prio else 0) for _ in range(S)]
        main = torch.cuda.current_stream()

        def run():
            for st in streams:
                st.wait_stream(main)
            for t in range(T):
                for s, e in enumerate(envs):
                    sl = slice(s * m, (s + 1) * m)
                    with torch.cuda.stream(streams[s]):
                        _native.check(lib.cf2_policy_forward(
                            fused.w.data_ptr(), m, 34, fused.prec, obs[t, sl].data_ptr(), fused.seed, t, s * m, 1,
                            act[t, sl].data_ptr(), val[t, sl].data_ptr(), lp[t, sl].data_ptr(),
                            streams[s].cuda_stream), "cf2_policy_forward")
                        e.step_into(act[t, sl], obs[t + 1, sl], rew[t, sl], d8[t, sl], t8[t, sl], final_obs_out=fin[t, sl])
            for st in streams:
                main.wait_stream(st)
        run()
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            obs[0] = obs[T]
            run()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps / T
        out.append({"shards": S, "us_per_env_step": dt * 1e6, "env_steps_per_s": args.envs / dt,
                    "checksum": float(obs[T].double().sum()), "prio": args.prio})
        print(json.dumps(out[-1]), flush=True)
        for e in envs:
            e.close()
        del obs, act, val, lp, rew, d8, t8, fin


if __name__ == "__main__":
    main()
