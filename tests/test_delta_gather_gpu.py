"""The delta observation exchange on the GPU (csrc/cf2sim_exchange.hip: cf2_obs_pack /
cf2_obs_consume / cf2_obs_rows): the kernels produce the torch-op version's ages and rows bit for
bit (partial blocks, several ranks, overflow), and with the product env the rows materialised on
request equal the full all-gather of the observation rows over 240 env-steps with auto-resets and
time-outs -- over one RCCL rank (the path of the 8-GPU run: eager per step, one C call per
env-step, and hipGraph units of 8 env-steps through cf2_xchg_run), through the process group's
all-gather, and over two gloo ranks sharing the test box's GPU."""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV_ID = "DroneHoverBulletFreeEnvWithGust-v0"


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _synthetic(world, n, ol, seed):
    """Every rank's rows of two consecutive steps, reset flags, ages and three steps' actions."""
    g = torch.Generator().manual_seed(seed)
    od = 2 * (ol + 4)
    N = world * n
    prev = torch.randn(N, od, generator=g)
    cur = torch.randn(N, od, generator=g)
    reset = (torch.rand(N, generator=g) < 0.06).to(torch.uint8)
    age = torch.randint(0, 6, (N,), generator=g, dtype=torch.int32)
    acts = [torch.randn(N, 4, generator=g) for _ in range(3)]
    return prev, cur, reset, age, acts


@pytest.mark.parametrize("world,n,ol,cap", [(1, 4096, 13, 307), (3, 1000, 13, 75), (2, 333, 17, 40),
                                             (2, 5000, 13, 10)])      # the last one overflows
def test_kernels_equal_torch_ops(gpu, world, n, ol, cap):
    from cf2sim.dist import consume_obs, obs_rows, pack_obs, packed_words
    prev, cur, reset, age, acts = _synthetic(world, n, ol, seed=world * 100 + n)
    words, wp = packed_words(n, ol, cap), packed_words(n, ol, 0)
    # pack: GPU per rank vs CPU per rank; the side-entry order differs (atomics), the rows must not
    pk_cpu = torch.cat([pack_obs(cur[r * n:(r + 1) * n], reset[r * n:(r + 1) * n], cap) for r in range(world)])
    pp_cpu = torch.cat([pack_obs(prev[r * n:(r + 1) * n], torch.zeros(n, dtype=torch.uint8), 0) for r in range(world)])
    pk_gpu = torch.empty(world * words, dtype=torch.int32, device=gpu)
    for r in range(world):
        pack_obs(cur[r * n:(r + 1) * n].to(gpu), reset[r * n:(r + 1) * n].to(gpu), cap, out=pk_gpu[r * words:(r + 1) * words])
    g = pk_gpu.cpu().view(world, words)
    c = pk_cpu.view(world, words)
    side = 4 + n * ol + (n + 31) // 32
    assert torch.equal(g[:, :side], c[:, :side]), "header, o_k rows and bitmap are deterministic"
    # consume
    age_c = age.clone()
    ovf_c = torch.zeros(1, dtype=torch.int32)
    pred_c = torch.ones(2, world, dtype=torch.int32)
    pred_c[0].zero_()
    consume_obs(pk_cpu, world, n, ol, cap, age_c, ovf_c, 4, pred_c[0], pred_c[1])
    age_g = age.to(torch.int16).to(gpu)                    # uint16 storage on the GPU
    ovf_g = torch.zeros(1, dtype=torch.int32, device=gpu)
    pred_g = torch.ones(2, world, dtype=torch.int32, device=gpu)
    pred_g[0].zero_()
    consume_obs(pk_gpu, world, n, ol, cap, age_g, ovf_g, 4, pred_g[0], pred_g[1])
    torch.cuda.synchronize()
    assert torch.equal(age_g.cpu().to(torch.int32) & 0xFFFF, age_c)
    assert (int(ovf_g.item()) > 0) == (int(ovf_c.item()) > 0)
    assert torch.equal(pred_g.cpu(), pred_c) and int(pred_c[0].sum()) > 0 and int(pred_c[1].sum()) == 0
    # rows: all of them, and a ragged window across a rank boundary
    out_c = obs_rows(pk_cpu, cap, pp_cpu, 0, world, n, ol, age_c, *acts)
    out_g = obs_rows(pk_gpu, cap, pp_cpu.to(gpu), 0, world, n, ol, age_g, *[a.to(gpu) for a in acts])
    r0, nr = max(0, n - 77), min(world * n - max(0, n - 77), 300)
    win_g = obs_rows(pk_gpu, cap, pp_cpu.to(gpu), 0, world, n, ol, age_g, *[a.to(gpu) for a in acts], row0=r0, nrows=nr)
    torch.cuda.synchronize()
    og = out_g.cpu()
    if cap != 10:
        assert torch.equal(og, out_c) and int(ovf_c.item()) == 0
    else:
        # overflow: the GPU and the CPU hand the slots to different blocks, so each drops other
        # blocks; every row neither marked is equal, and the marks sit on reset rows only
        ng, nc = torch.isnan(og).any(1), torch.isnan(out_c).any(1)
        both = ~ng & ~nc
        assert torch.equal(og[both], out_c[both]) and bool((ng <= reset.bool()).all())
        assert int(ovf_g.item()) > 0 and int(ng.sum()) > 0
    assert torch.equal(torch.nan_to_num(win_g.cpu(), 7.0), torch.nan_to_num(og[r0:r0 + nr], 7.0))


def test_overflow_nans_exactly_the_reset_rows_that_got_no_slot(gpu):
    """A rank with more resets than its side slab: in exactly the 64-env blocks its packed buffer
    marks dropped, the reset rows past the block's quota have NaN in o_0 / A; their o_k parts and
    every other row (the dropped blocks' first `quota` resets, that rank's other reset rows, the
    other rank's) are exactly the rows the history rules give, and the overflow count is the number
    of dropped blocks."""
    from cf2sim.dist import PACK_BLOCK, PACK_DROPPED, consume_obs, obs_rows, pack_obs, pack_quota, packed_words
    world, n, ol = 2, 3000, 13
    od = 2 * (ol + 4)
    prev, cur, _, age, acts = _synthetic(world, n, ol, seed=9)
    reset = torch.zeros(world * n, dtype=torch.uint8)
    reset[torch.arange(0, n, 7)] = 1              # rank 0: 429 resets
    reset[n + torch.arange(0, n, 97)] = 1         # rank 1: 31 resets
    cap = 100                                     # rank 0 overflows, rank 1 does not
    words = packed_words(n, ol, cap)
    pk = torch.empty(world * words, dtype=torch.int32, device=gpu)
    for r in range(world):
        pack_obs(cur[r * n:(r + 1) * n].to(gpu), reset[r * n:(r + 1) * n].to(gpu), cap, out=pk[r * words:(r + 1) * words])
    pp = torch.cat([pack_obs(prev[r * n:(r + 1) * n], torch.zeros(n, dtype=torch.uint8), 0) for r in range(world)]).to(gpu)
    age_g = age.to(torch.int16).to(gpu)
    ovf = torch.zeros(1, dtype=torch.int32, device=gpu)
    consume_obs(pk, world, n, ol, cap, age_g, ovf)
    rows = obs_rows(pk, cap, pp, 0, world, n, ol, age_g, *[a.to(gpu) for a in acts]).cpu()
    # the blocks each rank's pack marked dropped
    nb, nblk = (n + 31) // 32, (n + PACK_BLOCK - 1) // PACK_BLOCK
    pkc = pk.cpu().view(world, words)
    dropped_env = torch.zeros(world * n, dtype=torch.bool)
    ndrop = 0
    for r in range(world):
        bt = pkc[r, 4 + n * ol + nb:4 + n * ol + nb + nblk]
        d = bt == PACK_DROPPED
        ndrop += int(d.sum())
        dropped_env[r * n:(r + 1) * n] = d.repeat_interleave(PACK_BLOCK)[:n]
    assert int(ovf.item()) == ndrop > 0
    # the side slab is full: at most cap entries were placed, and no rank-1 block was dropped
    assert not bool(dropped_env[n:].any())
    # expected rows from the definitions (the env's rows of this step are `cur` where reset)
    a = (age.to(torch.int64) + 1).clamp(max=0xFFFF)
    a[reset.bool()] = 0
    exp = torch.empty(world * n, od)
    exp[:, :ol] = prev[:, ol + 4:2 * ol + 4]
    exp[:, ol:ol + 4] = torch.where((a >= 3)[:, None], acts[2], acts[0])
    exp[:, ol + 4:2 * ol + 4] = cur[:, ol + 4:2 * ol + 4]
    exp[:, 2 * ol + 4:] = torch.where((a == 1)[:, None], acts[0], acts[1])
    rs = reset.bool()
    exp[rs, :ol + 4] = cur[rs, :ol + 4]
    exp[rs, 2 * ol + 4:] = cur[rs, ol:ol + 4]
    # a dropped block keeps its first `quota` resets (their own slots); only the excess is lost
    rank = torch.zeros(world * n, dtype=torch.int64)
    for b0 in range(0, world * n, n):
        for s0 in range(b0, b0 + n, PACK_BLOCK):
            blk = rs[s0:min(s0 + PACK_BLOCK, b0 + n)].to(torch.int64)
            rank[s0:s0 + blk.numel()] = torch.cumsum(blk, 0) - blk
    q = pack_quota(n, cap)
    assert q == 2
    lost = rs & dropped_env & (rank >= q)
    assert 0 < int(lost.sum()) < int(rs[:n].sum()), "some, not all, of rank 0's reset rows are lost"
    assert not bool((rs & dropped_env & (rank < q)).logical_and(torch.isnan(rows).any(1)).any())
    nan_part = torch.zeros(world * n, od, dtype=torch.bool)
    nan_part[lost, :ol + 4] = True
    nan_part[lost, 2 * ol + 4:] = True
    assert bool(torch.isnan(rows[nan_part]).all()), "every reset row of a dropped block is marked"
    assert torch.equal(rows[~nan_part], exp[~nan_part]), "everything else is exact"


STANDIN = os.path.join(ROOT, "tests", "standin_rccl", "_build", "libstandin_rccl.so")


def _run_env(rank, world, port, out, backend, n, T, exchange="native", standin=False, fail_rank=-1):
    sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))
    os.environ["CF2SIM_EXCHANGE"] = "torch" if exchange == "torch" else "native"
    os.environ["CF2_STANDIN_FAIL_RANK"] = str(fail_rank)
    import torch.distributed as dist
    from cf2sim.dist import NO_WATCH, PipelinedObsGather, _pg_device, gather_rows
    from cf2sim.vec_env import BatchedCrazyflieEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    N = world * n
    env = BatchedCrazyflieEnv(ENV_ID, n, seed=3, env_id_offset=rank * n, device=dev, max_episode_steps=41)
    obs0 = env.reset().clone()
    # every env still flying at env-step 41 times out at once: the look-ahead (33 steps: the shortest
    # the batches of 16 allow, so the watch age 8 is inside the episode) sizes that step's capacity
    # from the receivers' counts, the other steps run at the 7.5 % crash budget (default_cap)
    # (the policy-in-the-loop runs crash up to ~10 % of the envs in one env-step, past the 7.5 %
    # default budget: a 25 % budget there; the quota stays that of the default budget)
    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=True, max_steps=41, lookahead=33,
                              cap=n // 4 if exchange == "step" else None, rccl_path=STANDIN if standin else None)
    assert pipe.watch != NO_WATCH and pipe.npred >= 33
    caps = []
    _after = pipe._after

    def _rec(k0, nb, cap, q, copied):
        caps.append(cap)
        return _after(k0, nb, cap, q, copied)
    pipe._after = _rec
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    ring = torch.rand(8, N, 4, device=dev, generator=g) * 2 - 1      # every rank holds every action
    acts = [ring[k % 8] for k in range(T)]
    slab = pipe.start(obs0)
    pipe.drain()
    bad, resets, checked = [], 0, 0
    full = gather_rows(obs0, sizes=[n] * world)
    if not torch.equal(slab, full):
        bad.append(-1)
    if not torch.equal(pipe.rows(acts[0], acts[0], acts[0]), full):
        bad.append(-2)

    def a3(k):
        return acts[k], acts[max(k - 1, 0)], acts[max(k - 2, 0)]

    if exchange == "run":
        # batches: a twin env steps the same actions eagerly for the reference rows
        twin = BatchedCrazyflieEnv(ENV_ID, n, seed=3, env_id_offset=rank * n, device=dev, max_episode_steps=41)
        twin.reset()
        ptrs = [ring[r][rank * n:(rank + 1) * n].data_ptr() for r in range(8)]
        k = 0
        for G in [16, 3, 5, 8] + [16] * ((T - 48) // 16) + [9, 7] if T == 240 else [16, 3, 5, 8] + [16] * ((T - 32) // 16):
            for s in range(G):
                twin.step_raw(ptrs[(k + s) % 8])
                resets += int(gather_rows(twin.done, sizes=[n] * world).sum())
            last = pipe.run(env, ptrs, G)
            k += G
            assert last == k - 1
            full = gather_rows(twin.obs, sizes=[n] * world)
            rows = pipe.rows(*a3(k - 1))
            checked += 1
            if not torch.equal(rows, full):
                bad.append(k - 1)
        twin.close()
    elif exchange == "step":
        # a policy in the loop: each action is computed from the local rows of the step before
        # (pipe.local_obs()), the exchange runs per batch; rows checked at irregular flushes
        twin = BatchedCrazyflieEnv(ENV_ID, n, seed=3, env_id_offset=rank * n, device=dev, max_episode_steps=41)
        twin.reset()
        side = torch.cuda.Stream(device=dev)          # steps issued from a pool stream, as step() advises
        side.wait_stream(torch.cuda.current_stream())
        taken = []
        with torch.cuda.stream(side):
            for k in range(T):
                loc = pipe.local_obs()
                if not torch.equal(loc, twin.obs if k > 0 else obs0):
                    bad.append(("local", k))
                a = (torch.tanh(3.0 * loc[:, 17:21]) * 0.5 + ring[k % 8][rank * n:(rank + 1) * n] * 0.5).contiguous()
                taken.append(a)
                twin.step_raw(a.data_ptr())
                resets += int(twin.done.sum())
                assert pipe.step(env, a.data_ptr()) == k
                if k % 7 == 6 or k == T - 1:
                    if k % 16 != 15:
                        try:
                            pipe.rows(a, a, a)
                            bad.append(("rows before flush", k))
                        except RuntimeError:
                            pass
                    pipe.flush()
                    ga = [gather_rows(taken[max(k - d, 0)], sizes=[n] * world) for d in range(3)]
                    rows = pipe.rows(*ga)
                    checked += 1
                    if not torch.equal(rows, gather_rows(twin.obs, sizes=[n] * world)):
                        bad.append(k)
        torch.cuda.current_stream().wait_stream(side)
        twin.close()
    else:
        for k in range(T):
            a = acts[k]
            j = pipe.k % pipe.depth
            if exchange == "native_env":       # env-step + exchange in one C call
                pipe.step_and_publish(env, a[rank * n:(rank + 1) * n].data_ptr())
            else:
                buf = pipe.buffer()
                done = pipe.done_buffer()
                env.step_raw(a[rank * n:(rank + 1) * n].data_ptr(), obs_ptr=buf.data_ptr(), done_ptr=done.data_ptr())
                pipe.publish()
            rows = pipe.rows(*a3(k))
            torch.cuda.synchronize()
            full = gather_rows(pipe.obs[j], sizes=[n] * world)
            resets += int(gather_rows(pipe.done[j], sizes=[n] * world).sum())
            checked += 1
            if not torch.equal(rows, full):
                bad.append(k)
    torch.cuda.synchronize()
    how = pipe.exchange
    ovf = pipe.overflows()
    pipe.close()
    # every rank's mismatches and overflows count (rank 0 writes the sums)
    tot = torch.tensor([len(bad), ovf], dtype=torch.int64, device=_pg_device(None, dev))
    dist.all_reduce(tot)
    if rank == 0:
        with open(out, "w") as f:
            f.write(f"{int(tot[0])} {resets} {int(tot[1])} {how} {checked} {len(set(caps))} {bad[:3]}")
    dist.destroy_process_group()


def _check(out, how, min_checked=200):
    nbad, resets, ovf, got, checked, ncaps = open(out).read().split()[:6]
    assert int(nbad) == 0, open(out).read()
    assert int(resets) > 0 and int(ovf) == 0
    assert got == how
    assert int(checked) >= min_checked
    # the side capacity varies: the crash budget, and the predicted time-outs at the TimeLimit steps
    assert int(ncaps) >= 2, open(out).read()


def test_delta_exchange_one_rccl_rank(gpu, tmp_path):
    """The native exchange, eager: cf2_xchg_publish per step (pack, our own RCCL communicator's
    all-gather, consume) and the rows materialised after every step."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 32768, 240), nprocs=1, join=True)
    _check(out, "native")


def test_delta_exchange_one_rccl_rank_env_step_in_one_call(gpu, tmp_path):
    """The native exchange's registered form: env-step + exchange per cf2_xchg_env_step call."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 32768, 240, "native_env"), nprocs=1, join=True)
    _check(out, "native")


def test_delta_exchange_one_rccl_rank_batched_run(gpu, tmp_path):
    """cf2_xchg_run: batches of env-steps with the pack fused in (cf2_step_packed), one RCCL
    all-gather and one consume per batch (units of 16, entered with partial batches of 3 and 5);
    the rows of each batch's last step equal the full gather of an eagerly stepped twin env's
    observations."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 32768, 240, "run"), nprocs=1, join=True)
    _check(out, "native", min_checked=16)


def test_delta_exchange_one_rccl_rank_policy_in_the_loop(gpu, tmp_path):
    """step(): the batch's env-steps issued one at a time, each action computed on the GPU from the
    local rows of the step before (local_obs(), equal to an eagerly stepped twin's every step), the
    exchange per batch of 16 or at irregular flush()es (every 7th step); rows() refuses to run over
    un-exchanged steps, and after each flush the rows equal the full gather of the twin's."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 32768, 240, "step"), nprocs=1, join=True)
    _check(out, "native", min_checked=30)


def _batch_misuse(rank, world, port, out):
    sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))
    os.environ["CF2SIM_EXCHANGE"] = "native"
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather
    from cf2sim.vec_env import BatchedCrazyflieEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    n = 4096
    env = BatchedCrazyflieEnv(ENV_ID, n, seed=3, device=dev)
    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=True, max_steps=500)
    pipe.start(env.reset().clone())
    lib, x = pipe._lib, pipe._xchg
    sp = torch.cuda.current_stream().cuda_stream
    a = torch.zeros(n, 4, device=dev)
    rew, trunc, cost, level = env._raw_step_outputs()
    res = []
    res.append(lib.cf2_xchg_step(x, env._ctx, a.data_ptr(), rew, trunc, cost, level, sp))   # no open batch
    res.append(lib.cf2_xchg_end(x, 0, None, sp))                                            # no open batch
    res.append(lib.cf2_xchg_begin(x, 64, 1, sp))                                            # not the next region
    res.append(lib.cf2_xchg_begin(x, 64, 0, sp))                                            # ok
    res.append(lib.cf2_xchg_begin(x, 64, 1, sp))                                            # already open
    res.append(lib.cf2_xchg_end(x, 0, None, sp))                                            # open, but no step yet
    res.append(lib.cf2_xchg_publish(x, 0, 64, 1, sp))                                       # a batch is open
    res.append(lib.cf2_xchg_step(x, env._ctx, a.data_ptr() + 4, rew, trunc, cost, level, sp))   # misaligned actions
    other = BatchedCrazyflieEnv(ENV_ID, 2 * n, seed=3, device=dev)
    res.append(lib.cf2_xchg_step(x, other._ctx, a.data_ptr(), rew, trunc, cost, level, sp))  # a shard of another size
    other.close()
    res.append(lib.cf2_xchg_step(x, env._ctx, a.data_ptr(), rew, trunc, cost, level, sp))   # ok
    res.append(lib.cf2_xchg_end(x, 0, None, sp))                                            # ok: exchanges step 0
    torch.cuda.synchronize()
    pipe._lib = None
    pipe._xchg = None
    lib.cf2_xchg_destroy(x)
    with open(out, "w") as f:
        f.write(" ".join(str(r) for r in res))
    dist.destroy_process_group()


def test_batch_calls_reject_misuse(gpu, tmp_path):
    """cf2_xchg_begin / cf2_xchg_step / cf2_xchg_end: a step or an end without an open batch, a
    begin on the wrong region or while a batch is open, an end with no step, a publish while a
    batch is open, misaligned actions and an env of another shard size return CF2_ERR_INVALID_ARG;
    the well-formed sequence
    returns CF2_OK."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_batch_misuse, args=(1, _port(), out), nprocs=1, join=True)
    got = [int(v) for v in open(out).read().split()]
    assert got == [-1, -1, -1, 0, -1, -1, -1, -1, -1, 0, 0], got


def test_delta_exchange_one_rccl_rank_batched_run_large_shard(gpu, tmp_path):
    """The same above 32 768 envs: the pack fused into step_kernel (256-env blocks, 4 pack blocks
    each, a ragged last block) instead of step_kernel_small."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 40000, 120, "run"), nprocs=1, join=True)
    _check(out, "native", min_checked=8)


def test_delta_exchange_one_rccl_rank_torch_path(gpu, tmp_path):
    """The same exchange with the process group's all-gather between the launches from Python."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 32768, 240, "torch"), nprocs=1, join=True)
    _check(out, "torch")


def test_delta_exchange_two_gloo_ranks_on_one_gpu(gpu, tmp_path):
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(2, _port(), out, "gloo", 4096, 240), nprocs=2, join=True)
    _check(out, "gloo")


def test_native_exchange_two_ranks_batched_run(gpu, tmp_path):
    """The native exchange at world size 2 (two processes sharing the box's GPU over a gloo group;
    the four RCCL entry points bound to the test stand-in, tests/standin_rccl): cf2_xchg_run's
    batches -- the [world][nb][words] receive layout with a rank stride of nb * words, both ranks'
    look-ahead counts agreeing on every step's capacity through ~6 TimeLimit periods -- give rows
    equal to the full gather of an eagerly stepped twin's observations after every batch, with no
    overflow, on both ranks."""
    assert os.path.exists(STANDIN), "build the stand-in first (tests/standin_rccl: make; __graft_entry__.build())"
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(2, _port(), out, "gloo", 4096, 240, "run", True), nprocs=2, join=True)
    _check(out, "native", min_checked=16)


def test_native_exchange_two_ranks_policy_in_the_loop(gpu, tmp_path):
    """The same two ranks through step() / flush(): the batch's env-steps issued one at a time from
    the local rows, the exchange at each batch end and at irregular flushes; rows equal at every
    flush on both ranks."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(2, _port(), out, "gloo", 4096, 240, "step", True), nprocs=2, join=True)
    _check(out, "native", min_checked=30)


def test_native_exchange_setup_failure_on_one_rank_falls_back_on_all(gpu, tmp_path):
    """Rank 1's communicator setup fails: the setup agreement makes both ranks fall back together
    (to the process group's exchange through the host) instead of leaving rank 0 in the native
    path, and the rows stay exact."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(2, _port(), out, "gloo", 4096, 96, "native", True, 1), nprocs=2, join=True)
    _check(out, "gloo", min_checked=96)


def test_rows_from_a_batched_receive_layout_with_rank_stride(gpu):
    """cf2_obs_rows on the batched receive layout [world][nb][words] built by hand (world 3, a
    batch of 4 steps, a ragged shard of 1000 envs): rank r's pack of step j sits at
    (r * nb + j) * words, so step j's rows read rank r at a stride of nb * words from j * words, and
    step j - 1's likewise.  Every step of the batch, whole and in a window spanning two ranks, equals
    the CPU restatement at the same stride bit for bit (NaN rows included: one block overflows)."""
    from cf2sim.dist import obs_rows, pack_obs, packed_words
    world, nb, n, ol, cap = 3, 4, 1000, 13, 75
    od = 2 * (ol + 4)
    words = packed_words(n, ol, cap)
    stride = nb * words
    g = torch.Generator().manual_seed(31)
    recv = torch.zeros(world * nb * words, dtype=torch.int32, device=gpu)
    for r in range(world):
        for j in range(nb):
            obs = torch.randn(n, od, generator=g)
            rs = (torch.rand(n, generator=g) < 0.06).to(torch.uint8)
            if r == 1 and j == 2:
                rs[128:192] = 1                     # a whole block resets: its excess overflows the spill area
            k = r * nb + j
            pack_obs(obs.to(gpu), rs.to(gpu), cap, out=recv[k * words:(k + 1) * words])
    torch.cuda.synchronize()
    recv_c = recv.cpu()
    N = world * n
    for j in range(1, nb):
        age = torch.randint(0, 6, (N,), generator=g, dtype=torch.int32)
        acts = [torch.randn(N, 4, generator=g) for _ in range(3)]
        for row0, nrows in ((0, N), (n - 7, n + 20)):
            want = obs_rows(recv_c[j * words:], cap, recv_c[(j - 1) * words:], cap, world, n, ol, age, *acts,
                            row0=row0, nrows=nrows, stride=stride, stride_prev=stride)
            got = obs_rows(recv[j * words:], cap, recv[(j - 1) * words:], cap, world, n, ol,
                           age.to(torch.int16).to(gpu), *[a.to(gpu) for a in acts],
                           row0=row0, nrows=nrows, stride=stride, stride_prev=stride)
            torch.testing.assert_close(got.cpu(), want, rtol=0, atol=0, equal_nan=True)
        assert torch.isnan(want).any() or j != 2, "step 2 of rank 1 overflowed"


def test_operands_the_kernels_would_overrun_are_rejected(gpu):
    """Host-side checks before the launch: a uint8 age vector (half the bytes the kernel indexes),
    short rows / packed buffers, or a pack whose next counters are its own raise ValueError instead
    of faulting on the device."""
    from cf2sim.dist import PACK_SCRATCH_WORDS, consume_obs, obs_rows, pack_obs, packed_words
    n, ol, cap = 256, 13, 16
    od = 2 * (ol + 4)
    prev = torch.zeros(n, od, device=gpu)
    a = torch.zeros(n, 4, device=gpu)
    pk = pack_obs(prev, torch.zeros(n, dtype=torch.uint8, device=gpu), cap)
    good_age = torch.zeros(n, dtype=torch.int16, device=gpu)
    consume_obs(pk, 1, n, ol, cap, good_age)
    obs_rows(pk, cap, pk, cap, 1, n, ol, good_age, a, a, a)
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        consume_obs(pk, 1, n, ol, cap, torch.zeros(n, dtype=torch.uint8, device=gpu))
    with pytest.raises(ValueError):
        obs_rows(pk, cap, pk, cap, 1, n, ol, good_age, a, a, a, out=torch.empty(n // 2, od, device=gpu))
    with pytest.raises(ValueError):
        obs_rows(pk[: packed_words(n, ol, cap) // 2], cap, pk, cap, 1, n, ol, good_age, a, a, a)
    with pytest.raises(ValueError):
        pack_obs(prev, torch.zeros(n, dtype=torch.uint8, device=gpu), cap, out=torch.zeros(8, dtype=torch.int32, device=gpu))
    scr = torch.zeros(PACK_SCRATCH_WORDS, dtype=torch.int32, device=gpu)
    with pytest.raises(ValueError):
        pack_obs(prev, torch.zeros(n, dtype=torch.uint8, device=gpu), cap, out=pk, scratch=scr, next_scratch=scr)
