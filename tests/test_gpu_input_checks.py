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


def _tables(t, gpu):
    ax = torch.linspace(-1.0, 1.0, 15, device=gpu)
    g = [ax.view([-1 if i == d else 1 for i in range(6)]) for d in range(6)]
    return torch.stack([sum((0.3 + 0.1 * k + 0.05 * d) * g[d] ** (1 + (d + k) % 2) for d in range(6))
                        + 0.1 * torch.sin(3 * g[3] + 2 * g[4] - g[5] + k) for k in range(t)]).reshape(t, -1)


def test_bind_tables_written_on_a_side_stream(gpu):
    """cf2_bind_hj_tables derives the sign bits from V after all device work (it used to
    run on the null stream, unordered with a torch side stream still writing V).  V is produced on a
    side stream behind a long queue of work and bound without any host synchronisation; the env
    then steps exactly like one bound to a V that was complete before binding."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env_id, n = "DroneHoverBulletFreeEnvWithAdversary-v0", 2048
    ref_V = _tables(1, gpu)
    torch.cuda.synchronize()
    ref = BatchedCrazyflieEnv(env_id, n, seed=5)
    ref.bind_hj_tables(ref_V)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        V = torch.zeros(1, 15 ** 6, device=gpu)
        x = torch.randn(2048, 2048, device=gpu)
        for _ in range(40):                        # keep the side stream busy before V is written
            x = torch.tanh(x @ x * 1e-3)
        V.copy_(ref_V + 0.0 * x[0, 0])
    env = BatchedCrazyflieEnv(env_id, n, seed=5)
    env.bind_hj_tables(V)                          # no synchronisation with `side` by the caller
    torch.cuda.current_stream().wait_stream(side)
    env.reset()
    ref.reset()
    gen = torch.Generator(device=gpu)
    gen.manual_seed(1)
    for _ in range(20):
        a = torch.rand(n, 4, device=gpu, generator=gen) * 0.3
        o1, r1, _, _ = env.step(a)
        o2, r2, _, _ = ref.step(a)
        assert torch.equal(o1, o2) and torch.equal(r1, r2)
    env.close()
    ref.close()


def test_rebinding_tables(gpu):
    """Rebinding grows the sign-bit buffer when more tables are bound; a rejected binding (a level
    mapped past the bound tables) leaves the previous one in place."""
    from cf2sim import _native
    from cf2sim.vec_env import BatchedCrazyflieEnv
    env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithRandomHJAdversary-v0", 512, seed=2)
    nl = int(env.cfg.num_levels)
    env.bind_hj_tables(_tables(1, gpu), table_of_level=[0] * nl)
    env.bind_hj_tables(_tables(3, gpu), table_of_level=[k % 3 for k in range(nl)])   # larger: new buffer
    env.reset()
    env.step(torch.zeros(512, 4, device=gpu))
    with pytest.raises(_native.CF2Error):
        env.bind_hj_tables(_tables(2, gpu), table_of_level=[2] * nl)    # row 2 of 2 tables
    env.step(torch.zeros(512, 4, device=gpu))                            # previous binding still valid
    torch.cuda.synchronize()
    env.close()


def test_hbm_probe(gpu):
    """cf2_hbm_probe (bench.py's HBM-rate probe): exact copy with a ragged tail, the read mode
    leaves dst alone, argument checks."""
    from cf2sim import _native
    lib = _native.load()
    s = torch.cuda.current_stream().cuda_stream
    src = torch.arange(1_000_004, dtype=torch.float32, device="cuda")      # 4 000 016 B: 16-B multiple
    dst = torch.zeros_like(src)
    assert lib.cf2_hbm_probe(dst.data_ptr(), src.data_ptr(), src.numel() * 4, 0, s) == 0
    torch.cuda.synchronize()
    assert torch.equal(src, dst)
    sink = torch.zeros(1024, dtype=torch.float32, device="cuda")
    assert lib.cf2_hbm_probe(sink.data_ptr(), src.data_ptr(), src.numel() * 4, 1, s) == 0
    torch.cuda.synchronize()
    assert lib.cf2_hbm_probe(dst.data_ptr(), src.data_ptr(), 10, 0, s) != 0            # not a 16-B multiple
    assert lib.cf2_hbm_probe(dst.data_ptr() + 4, src.data_ptr(), 16, 0, s) != 0        # misaligned
    assert lib.cf2_hbm_probe(None, src.data_ptr(), 16, 0, s) != 0
    assert lib.cf2_hbm_probe(dst.data_ptr(), src.data_ptr(), 16, 2, s) != 0            # no such mode


def test_step_output_buffers_and_copy(gpu):
    """step() returns the env's own output buffers (documented: the next step overwrites them);
    step(copy=True) / copy_outputs=True return fresh tensors that later steps leave alone."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = 256
    env = BatchedCrazyflieEnv(ENV, n, seed=2)
    env.reset()
    a = torch.rand(n, 4, device=gpu) * 0.6 - 0.1
    o1, r1, d1, i1 = env.step(a)
    o2, r2, d2, i2 = env.step(a)
    assert o1 is o2 and r1 is r2 and d1 is d2 and i1["cost"] is i2["cost"]      # persistent buffers
    c1 = env.step(a, copy=True)
    keep = c1[0].clone()
    c2 = env.step(a, copy=True)
    assert c1[0] is not c2[0] and c1[0] is not env.obs
    assert torch.equal(c1[0], keep), "a copied result must not change with the next step"
    assert not torch.equal(c1[0], c2[0]), "two consecutive steps give different observations"
    env2 = BatchedCrazyflieEnv(ENV, n, seed=2, copy_outputs=True)
    env2.reset()
    x1, x2 = env2.step(a), env2.step(a)
    assert x1[0] is not x2[0] and x1[3]["cost"] is not x2[3]["cost"]
    env.close()
    env2.close()


def test_masked_reset_after_raw_obs_pointer_is_refused(gpu):
    """after a step into a raw obs pointer, a masked reset cannot produce the other envs'
    observations; it raises instead of returning stale rows."""
    from cf2sim.vec_env import BatchedCrazyflieEnv
    n = 128
    env = BatchedCrazyflieEnv(ENV, n)
    env.reset()
    a = torch.zeros(n, 4, device=gpu)
    raw = torch.empty(n, env.obs_dim, device=gpu)
    env.step_raw(a.data_ptr(), obs_ptr=raw.data_ptr())
    m = torch.zeros(n, dtype=torch.uint8, device=gpu)
    m[:3] = 1
    with pytest.raises(ValueError):
        env.reset(m)
    env.reset()              # a full reset is fine
    env.reset(m)             # and masked resets after it
    env.close()
