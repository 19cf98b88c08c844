"""Where do two launch geometries of the same envs differ?  Steps N envs in one context and in two
contexts of N/2 (global ids continued) with the same actions and lists, per env-step, the obs
components that are not bit-identical and whether the env reset in that step.
python tools/kernel_diff.py [--envs N] [--steps T] [--env-id ID]"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=262144)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--env-id", default="DroneHoverBulletFreeEnvWithGust-v0")
    ap.add_argument("--parts", type=int, default=2)
    args = ap.parse_args()
    from cf2sim.vec_env import BatchedCrazyflieEnv
    N, S = args.envs, args.parts
    full = BatchedCrazyflieEnv(args.env_id, N, seed=3)
    parts = [BatchedCrazyflieEnv(args.env_id, N // S, seed=3, env_id_offset=k * (N // S)) for k in range(S)]
    o1 = full.reset().cpu().numpy()
    o2 = np.concatenate([p.reset().cpu().numpy() for p in parts])
    print("reset obs mismatches:", int((o1 != o2).sum()))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11)
    total = 0
    for t in range(args.steps):
        a = (torch.rand(N, 4, device="cuda", generator=gen) * 2 - 1).contiguous()
        g1, r1, d1, _ = full.step(a)
        outs = [p.step(a[k * (N // S):(k + 1) * (N // S)].contiguous()) for k, p in enumerate(parts)]
        g1, d1 = g1.cpu().numpy(), d1.cpu().numpy().astype(bool)
        g2 = np.concatenate([o[0].cpu().numpy() for o in outs])
        bad = np.argwhere(g1 != g2)
        total += len(bad)
        for e, c in bad[:12]:
            print(f"step {t} env {e} comp {c} full {g1[e, c]!r} parts {g2[e, c]!r} reset {bool(d1[e])} "
                  f"region {'small' if e >= 196608 else 'large'}")
        s1 = full.get_state()[0].cpu().numpy()
        s2 = np.concatenate([p.get_state()[0].cpu().numpy() for p in parts], axis=1)
        nb = int((s1 != s2).sum())
        if nb:
            fb = np.argwhere(s1 != s2)
            print(f"step {t}: state mismatches {nb}, first fields {sorted(set(int(f) for f, _ in fb[:50]))}")
    print("total obs mismatches:", total)


if __name__ == "__main__":
    main()
