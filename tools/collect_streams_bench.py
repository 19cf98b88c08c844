"""Collect loop at N envs split into S contexts (shards of consecutive global env ids) whose
per-step launches go to S HIP streams, so that one shard's env-step can overlap another shard's
policy forward on the GPU.  Per env-step time (HIP events around --steps loop iterations after a
random-action warm-up) for each split and launch style:
  fused  -- cf2_collect_step per shard and step (env-step + policy in one launch)
  pair   -- cf2_step + cf2_policy_forward per shard and step
  roll   -- cf2_collect_rollout per shard, K = --steps env-steps in one launch
Results do not depend on the split (physics keyed by the global env id, the policy's noise by
row_offset = env_id_offset; tests/test_collect_fused.py::test_collect_is_split_invariant).
Prints one JSON line per configuration."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=600)
    ap.add_argument("--splits", default="1,2,4")
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    args = ap.parse_args()
    from cf2sim.rollout import FusedActorCritic, MLPActorCritic
    from cf2sim.vec_env import BatchedCrazyflieEnv
    N, T = args.envs, args.steps
    torch.manual_seed(0)
    ac = MLPActorCritic(obs_dim=34).cuda()
    for S in [int(x) for x in args.splits.split(",")]:
        n = N // S
        streams = [torch.cuda.Stream() for _ in range(S)]
        shards = []
        for s in range(S):
            with torch.cuda.stream(streams[s]):
                e = BatchedCrazyflieEnv(args.env_id, n, seed=0, env_id_offset=s * n, want_final_obs=True)
                p = FusedActorCritic(ac, seed=0, precision="bf16x3")
                e.reset()
                wa = torch.rand(8, n, 4, device="cuda") * 2 - 1
                for k in range(args.warmup):
                    e.step_raw(wa[k % 8].data_ptr())
                buf = {"act": torch.rand(T + 1, n, 4, device="cuda") * 2 - 1, "obs": torch.empty(T, n, 34, device="cuda"),
                       "fin": torch.empty(T, n, 34, device="cuda"), "rew": torch.empty(T, n, device="cuda"),
                       "val": torch.empty(T + 1, n, device="cuda"), "lp": torch.empty(T + 1, n, device="cuda"),
                       "d": torch.empty(T, n, dtype=torch.uint8, device="cuda"),
                       "tr": torch.empty(T, n, dtype=torch.uint8, device="cuda")}
                shards.append((e, p, buf))
        torch.cuda.synchronize()

        def run(style):
            if style == "roll":
                for s, (e, p, b) in enumerate(shards):
                    with torch.cuda.stream(streams[s]):
                        assert e.collect_rollout_into(b["act"], b["obs"], b["rew"], b["d"], b["tr"], b["fin"], p,
                                                      b["val"], b["lp"])
                return
            for t in range(T):
                for s, (e, p, b) in enumerate(shards):
                    with torch.cuda.stream(streams[s]):
                        if style == "fused":
                            assert e.collect_step_raw(b["act"][t].data_ptr(), b["obs"][t].data_ptr(), b["rew"][t].data_ptr(),
                                                      b["d"][t].data_ptr(), b["tr"][t].data_ptr(), b["fin"][t].data_ptr(),
                                                      p, b["act"][t + 1].data_ptr(), b["val"][t + 1].data_ptr(),
                                                      b["lp"][t + 1].data_ptr())
                        else:
                            e.step_into(b["act"][t], b["obs"][t], b["rew"][t], b["d"][t], b["tr"][t],
                                        final_obs_out=b["fin"][t])
                            p.step_into(b["obs"][t], b["act"][t + 1], b["val"][t + 1], b["lp"][t + 1],
                                        row_offset=int(e.cfg.env_id_offset))

        for style in ("fused", "pair", "roll"):
            run(style)                                   # warm-up of this style
            torch.cuda.synchronize()
            reps = 3
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(torch.cuda.current_stream())
            for st in streams:
                st.wait_event(e0)
            for _ in range(reps):
                run(style)
            for st in streams:
                ev = torch.cuda.Event()
                ev.record(st)
                torch.cuda.current_stream().wait_event(ev)
            e1.record(torch.cuda.current_stream())
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / (reps * T)
            print(json.dumps({"envs": N, "splits": S, "style": style, "us_per_env_step": us, "steps": T}), flush=True)
        for e, _, _ in shards:
            e.close()
        del shards


if __name__ == "__main__":
    main()
