"""Diagnostic (not collected by pytest): one fused collect step against cf2_step + cf2_policy_forward
from the same state, env part and policy part compared separately; then the first differing step
of a collect."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "disturbance-crazyfile-simulation_amd"))
from test_collect_fused import _pair  # noqa: E402


def d(a, b):
    return (a.float() - b.float()).abs().max().item(), int((a != b).sum().item())


def main():
    (ea, pa), (eb, pb) = _pair("DroneHoverBulletFreeEnvWithGust-v0", 40000, {})
    n, od, dev = ea.num_envs, ea.obs_dim, ea.device
    ea.reset(); eb.reset()
    g = torch.Generator(device=dev).manual_seed(1)
    for k in range(30):
        a = torch.rand(n, 4, device=dev, generator=g) * 2 - 1
        z = lambda *s, dt=torch.float32: torch.empty(*s, device=dev, dtype=dt)
        oa, ra, da, ta, fa, aa, va, la = z(n, od), z(n), z(n, dt=torch.uint8), z(n, dt=torch.uint8), z(n, od), z(n, 4), z(n), z(n)
        ob, rb, db, tb, fb, ab, vb, lb = z(n, od), z(n), z(n, dt=torch.uint8), z(n, dt=torch.uint8), z(n, od), z(n, 4), z(n), z(n)
        assert ea.collect_step_into(a, oa, ra, da, ta, fa, pa, aa, va, la)
        eb.step_into(a, ob, rb, db, tb, final_obs_out=fb)
        pb.step_into(ob, ab, vb, lb)
        torch.cuda.synchronize()
        print(k, "obs", d(oa, ob), "rew", d(ra, rb), "done", d(da, db), "act", d(aa, ab), "val", d(va, vb), "logp", d(la, lb))
        # policy alone on the fused kernel's observations
        ac2, vc2, lc2 = z(n, 4), z(n), z(n)
        pa.counter -= 1
        pa.step_into(oa, ac2, vc2, lc2)
        torch.cuda.synchronize()
        print("   policy_kernel on fused obs vs fused policy: act", d(aa, ac2), "val", d(va, vc2), "logp", d(la, lc2))
        bad = (aa != ac2).any(1).nonzero().flatten()
        if len(bad):
            r = bad[0].item()
            print("   first bad row", r, "row%256", r % 256, "rows bad", len(bad), aa[r].tolist(), ac2[r].tolist())
        if k >= 3:
            break


if __name__ == "__main__":
    main()
