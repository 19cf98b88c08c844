"""The fused collect paths must equal the two launches per env-step (cf2_step +
cf2_policy_forward) bit for bit -- observations, actions, values, log-probabilities, rewards,
flags, final observations, the GAE outputs and the env state afterwards -- across auto-resets,
time-outs, a partial last block, several residency slices and the HJ path:
  * cf2_collect_rollout: all K steps of the loop in one launch (collect_rollout_kernel);
  * cf2_collect_step: one launch per env-step (collect_kernel / collect_kernel_small).
Configs without a fused instance must fall back to the two launches.
The collect loop being restated is IWPGAlgorithm.roll_out (algs/iwpg/iwpg.py:372-410)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = [
    ("DroneHoverBulletFreeEnvWithGust-v0", 40000, {}),                                    # bench workload, partial block
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", 33024, dict(max_episode_steps=7, domain_randomization=0)),
    ("DroneHoverBulletFreeEnvWithRandomAdversary-v0", 65536, dict(max_episode_steps=11)),
    # small N (collect_kernel_small: 64 envs per block with helper waves)
    ("DroneHoverBulletFreeEnvWithGust-v0", 32768, {}),                                    # the 8-GPU node shard
    ("DroneHoverBulletFreeEnvWithConstWind-v0", 4096, dict(max_episode_steps=9)),         # C2
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", 5000, dict(domain_randomization=0)),   # partial last block
]


def _pair(env_id, n, kw, setup=None, count=2):
    from cf2sim.rollout import FusedActorCritic, MLPActorCritic
    from cf2sim.vec_env import BatchedCrazyflieEnv
    envs = [BatchedCrazyflieEnv(env_id, n, seed=11, want_final_obs=True, **kw) for _ in range(count)]
    torch.manual_seed(5)
    ac = MLPActorCritic(obs_dim=envs[0].obs_dim).cuda()
    with torch.no_grad():                    # non-trivial standardisation, as after a few epochs
        ac.obs_oms.mean.uniform_(-0.2, 0.2)
        ac.obs_oms.std.uniform_(0.5, 2.0)
        ac.ret_oms.std.fill_(3.0)
    out = []
    for e in envs:
        if setup is not None:
            setup(e)
        out.append((e, FusedActorCritic(ac, seed=7, precision="bf16x3")))
    return out


def _check_equal(ra, rb):
    for f in ("obs", "act", "rew", "val", "logp", "done", "trunc", "adv", "ret", "last_obs", "last_val", "trunc_val",
              "discounted_ret"):
        a, b = getattr(ra, f), getattr(rb, f)
        assert torch.equal(a, b), f"{f}: max |diff| {(a.float() - b.float()).abs().max().item()}"


def _spy(env, name, log):
    orig = getattr(env, name)

    def spy(*args, **kwargs):
        ok = orig(*args, **kwargs)
        log.append(ok)
        return ok
    setattr(env, name, spy)


def _run(env_id, n, kw, setup=None, T=24):
    """One collect per mode (one launch / one launch per step / two launches per step) from the
    same state; returns the fused calls' support flags (rollout, per-step)."""
    from cf2sim.rollout import collect
    (ea, pa), (es, ps), (eb, pb) = _pair(env_id, n, kw, setup, count=3)
    oa, os_, ob = ea.reset(), es.reset(), eb.reset()
    launched_roll, launched_step = [], []
    _spy(ea, "collect_rollout_into", launched_roll)
    _spy(es, "collect_step_into", launched_step)
    ra = collect(ea, pa, T, obs=oa.clone(), fuse=True)
    rs_ = collect(es, ps, T, obs=os_.clone(), fuse="steps")
    rb = collect(eb, pb, T, obs=ob.clone(), fuse=False)
    torch.cuda.synchronize()
    assert rb.done.any(), "no auto-reset inside the window"
    _check_equal(ra, rb)
    _check_equal(rs_, rb)
    gb, ib = eb.get_state()
    for e in (ea, es):
        g, i = e.get_state()
        assert torch.equal(i, ib) and torch.equal(g, gb)
    assert pa.counter == pb.counter == ps.counter
    # a second collect continues from the first one's last observation
    ra2 = collect(ea, pa, 5, obs=ra.last_obs, fuse=True)
    rs2 = collect(es, ps, 5, obs=rs_.last_obs, fuse="steps")
    rb2 = collect(eb, pb, 5, obs=rb.last_obs, fuse=False)
    _check_equal(ra2, rb2)
    _check_equal(rs2, rb2)
    # a collect that re-uses an earlier rollout's storage (out=) gives the same results
    ra3 = collect(ea, pa, 5, obs=ra2.last_obs, fuse=True, out=ra2)
    rb3 = collect(eb, pb, 5, obs=rb2.last_obs, fuse=False)
    assert ra3.storage is ra2.storage
    _check_equal(ra3, rb3)
    for e in (ea, es, eb):
        e.close()
    return launched_roll, launched_step


@pytest.mark.parametrize("env_id,n,kw", CASES)
def test_fused_collect_equals_two_launches(gpu, env_id, n, kw):
    roll, step = _run(env_id, n, kw)
    assert roll and all(roll) and step and all(step), "a fused kernel did not run"


def test_collect_rollout_over_several_slices(gpu):
    """More blocks than one residency round holds: cf2_collect_rollout runs the envs in slices."""
    roll, step = _run("DroneHoverBulletFreeEnvWithGust-v0", 200000, dict(max_episode_steps=5), T=7)
    assert roll and all(roll) and step and all(step)


def test_fused_collect_hj_boltzmann(gpu):
    from test_gpu_parity import _synthetic_tables
    V = torch.from_numpy(_synthetic_tables(tuple(range(3)), seed=1)).cuda()
    tol = [lv % 3 for lv in range(21)]
    roll, step = _run("DroneHoverBulletFreeEnvWithRandomHJAdversary-v0", 40000, dict(max_episode_steps=6),
                      setup=lambda e: e.bind_hj_tables(V, tol), T=12)
    assert roll and all(roll) and step and all(step)


@pytest.mark.parametrize("env_id,n,kw", [
    ("DroneHoverBulletFreeEnvWithGust-v0", 40000, dict(observation_noise=0)),  # 42-wide obs
    ("DroneHoverBulletFreeEnvWithGust-v0", 4096, dict(observation_noise=0)),   # 42-wide obs, small N
    ("DroneHoverSimpleEnv-v0", 40000, {}),
])
def test_unfused_configs_fall_back(gpu, env_id, n, kw):
    roll, step = _run(env_id, n, kw, T=8)
    assert roll == [False] * 3 and step == [False] * 2, \
        "an unsupported config launches nothing and is probed once per collect"


def test_collect_step_rejects_bad_args(gpu):
    from cf2sim import _native
    (e, p), _ = _pair("DroneHoverBulletFreeEnvWithGust-v0", 40000, {})
    n, d = e.num_envs, e.obs_dim
    e.reset()
    a = torch.zeros(n, 4, device=gpu)
    o = torch.empty(n, d, device=gpu)
    r = torch.empty(n, device=gpu)
    dn = torch.empty(n, dtype=torch.uint8, device=gpu)
    v, lp = torch.empty(n, device=gpu), torch.empty(n, device=gpu)
    with pytest.raises(ValueError):           # wrong shape of the next actions
        e.collect_step_into(a, o, r, dn, None, None, p, torch.empty(n, 3, device=gpu), v, lp)
    st = e.lib.cf2_collect_step(e._ctx, a.data_ptr(), o.data_ptr(), r.data_ptr(), dn.data_ptr(), None, None,
                                p.w.data_ptr(), d, p.prec, 0, 0, 0, a.data_ptr(), v.data_ptr(), lp.data_ptr(), e.stream)
    assert st != 0, "act_out aliasing act must be rejected"
    st = e.lib.cf2_collect_step(e._ctx, a.data_ptr(), o.data_ptr(), r.data_ptr(), dn.data_ptr(), None, None,
                                p.w.data_ptr(), d + 8, p.prec, 0, 0, 0, torch.empty(n, 4, device=gpu).data_ptr(),
                                v.data_ptr(), lp.data_ptr(), e.stream)
    assert st != 0 and st != _native.CF2_ERR_UNSUPPORTED, "an obs_dim that is not the env's is an error"
    # cf2_collect_rollout: K < 1, misaligned actions and a wrong obs_dim are errors, nothing launched
    K = 3
    A = torch.zeros(K + 1, n, 4, device=gpu)
    O = torch.empty(K, n, d, device=gpu)
    R, V, L = torch.empty(K, n, device=gpu), torch.empty(K + 1, n, device=gpu), torch.empty(K + 1, n, device=gpu)
    D = torch.empty(K, n, dtype=torch.uint8, device=gpu)
    args = lambda k, a, od: (e._ctx, k, a, O.data_ptr(), R.data_ptr(), D.data_ptr(), None, None, p.w.data_ptr(), od,
                             p.prec, 0, 0, 0, V.data_ptr(), L.data_ptr(), e.stream)
    for bad in (args(0, A.data_ptr(), d), args(K, A.data_ptr() + 4, d), args(K, A.data_ptr(), d + 8)):
        st = e.lib.cf2_collect_rollout(*bad)
        assert st != 0 and st != _native.CF2_ERR_UNSUPPORTED
    with pytest.raises(ValueError):           # act needs K + 1 slabs
        e.collect_rollout_into(A[:K], O, R, D, None, None, p, V, L)
    e.close()


@pytest.mark.parametrize("env_id,n,kw", [
    ("DroneHoverBulletFreeEnvWithGust-v0", 65536, {}),                                    # halves at small N
    ("DroneHoverBulletFreeEnvWithoutAdversary-v0", 8192, dict(max_episode_steps=9)),
])
def test_collect_is_split_invariant(gpu, env_id, n, kw):
    """A collect over two contexts holding global env ids [0, n/2) and [n/2, n) equals one collect
    over all n envs, env for env (physics keyed by the global env id through env_id_offset, the
    policy's sampling noise through row_offset = env_id_offset): rank-count invariance of f3."""
    from cf2sim.rollout import FusedActorCritic, MLPActorCritic, collect
    from cf2sim.vec_env import BatchedCrazyflieEnv
    torch.manual_seed(5)
    ac = MLPActorCritic(obs_dim=34).cuda()
    with torch.no_grad():
        ac.obs_oms.mean.uniform_(-0.2, 0.2)
        ac.obs_oms.std.uniform_(0.5, 2.0)
    h = n // 2
    whole = BatchedCrazyflieEnv(env_id, n, seed=3, want_final_obs=True, **kw)
    parts = [BatchedCrazyflieEnv(env_id, h, seed=3, env_id_offset=k * h, want_final_obs=True, **kw) for k in range(2)]
    rw = collect(whole, FusedActorCritic(ac, seed=9), 16)
    rp = [collect(e, FusedActorCritic(ac, seed=9), 16) for e in parts]
    torch.cuda.synchronize()
    assert rw.done.any()
    assert whole.last_collect_fused and all(e.last_collect_fused for e in parts)
    for f in ("obs", "act", "rew", "val", "logp", "done", "trunc", "adv", "ret", "last_obs", "last_val", "trunc_val"):
        a = getattr(rw, f)
        b = torch.cat([getattr(r, f) for r in rp], dim=1 if a.dim() >= 2 and a.shape[0] == 16 else 0)
        assert torch.equal(a, b), f"{f}: max |diff| {(a.float() - b.float()).abs().max().item()}"
    for e in [whole] + parts:
        e.close()
