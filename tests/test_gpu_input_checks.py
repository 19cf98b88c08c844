"""The host mirror checks every buffer before it reaches the kernel (the kernel trusts pointers and
sizes): wrong shape, dtype, device, contiguity or alignment raise ValueError in step(), step_into()
and bind_hj_tables(), never a GPU fault.  A Boltzmann-level env (one level drawn per episode,
envs/hover_free.py via distur_gener.py:155, which loads fastrack_{level}_15x15.npy per level) refuses
a single bound table unless the level map is given explicitly."""
import pytest
import torch

pytestmark = pytest.mark.gpu

ENV = "DroneHoverBulletFreeEnvWithoutAdversary-v0"


def _bufs(n, od, gpu):
    return dict(obs_out=torch.zeros(n, od, device=gpu), rew_out=torch.zeros(n, device=gpu),
                done_out=torch.zeros(n, dtype=torch.uint8, device=gpu))


def test_step_into_rejects_bad_buffers(gpu):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = 64
    env = BatchedCrazyflieEnv(ENV, n)
    env.reset()
    od = env.obs_dim
    a = torch.zeros(n, 4, device=gpu)
    env.step_into(a, **_bufs(n, od, gpu))                 # the well-formed call goes through
    bad = [
        (torch.zeros(n, 4, device=gpu, dtype=torch.float64), {}),             # action dtype
        (torch.zeros(n, 2, device=gpu), {}),                                  # action shape
        (torch.zeros(4, n, device=gpu).t(), {}),                              # not contiguous
        (torch.zeros(n, 4), {}),                                              # host tensor
        (torch.zeros(n * 4 + 1, device=gpu)[1:].view(n, 4), {}),              # misaligned
        (a, dict(obs_out=torch.zeros(n - 1, od, device=gpu))),                # undersized obs
        (a, dict(rew_out=torch.zeros(n, device=gpu, dtype=torch.float16))),   # reward dtype
        (a, dict(done_out=torch.zeros(n, device=gpu))),                       # done must be uint8
        (a, dict(trunc_out=torch.zeros(n, 2, dtype=torch.uint8, device=gpu))),
        (a, dict(cost_out=torch.zeros(n + 1, device=gpu))),
        (a, dict(final_obs_out=torch.zeros(n, od - 1, device=gpu))),
    ]
    for act, over in bad:
        kw = _bufs(n, od, gpu)
        kw.update(over)
        with pytest.raises(ValueError):
            env.step_into(act, **kw)
    with pytest.raises(ValueError):
        env.step(torch.zeros(n, 3, device=gpu))
    with pytest.raises(ValueError):
        env.step(torch.zeros(n + 1, 4, device=gpu))
    torch.cuda.synchronize()
    env.close()


def test_boltzmann_env_needs_one_table_per_level(gpu):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithRandomHJAdversary-v0", 64)
    nl = int(env.cfg.num_levels)
    V = torch.zeros(1, 15 ** 6, device=gpu)
    with pytest.raises(ValueError):
        env.bind_hj_tables(V)                              # one table for nl levels, no explicit map
    with pytest.raises(ValueError):
        env.bind_hj_tables(V, table_of_level=[0] * (nl - 1))
    with pytest.raises(ValueError):
        env.bind_hj_tables(torch.zeros(1, 15 ** 5, device=gpu), table_of_level=[0] * nl)
    env.bind_hj_tables(V, table_of_level=[0] * nl)        # an explicit map is accepted
    env.reset()
    env.step(torch.zeros(64, 4, device=gpu))
    torch.cuda.synchronize()
    env.close()
