"""The delta observation exchange on the GPU (csrc/cf2sim_exchange.hip, cf2_obs_pack /
cf2_obs_unpack): the kernels produce the torch-op version's rows bit for bit (partial blocks,
several ranks, overflow), and with the product env the rebuilt slab equals the full all-gather of
the observation rows over 240 env-steps with auto-resets and time-outs -- over one RCCL rank (the
path of the 8-GPU run) and over two gloo ranks sharing the test box's GPU."""
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
    """Every rank's rows of one step and the previous slab, with the history rules applied."""
    g = torch.Generator().manual_seed(seed)
    od = 2 * (ol + 4)
    N = world * n
    prev = torch.randn(N, od, generator=g)
    cur = torch.randn(N, od, generator=g)
    reset = (torch.rand(N, generator=g) < 0.06).to(torch.uint8)
    age = torch.randint(0, 6, (N,), generator=g, dtype=torch.int32)
    a_k, a_p = torch.randn(N, 4, generator=g), torch.randn(N, 4, generator=g)
    return prev, cur, reset, age, a_k, a_p


@pytest.mark.parametrize("world,n,ol,cap", [(1, 4096, 13, 307), (3, 1000, 13, 75), (2, 333, 17, 40),
                                             (2, 5000, 13, 10)])      # the last one overflows
def test_kernels_equal_torch_ops(gpu, world, n, ol, cap):
    from cf2sim.dist import pack_obs, packed_words, unpack_obs
    prev, cur, reset, age, a_k, a_p = _synthetic(world, n, ol, seed=world * 100 + n)
    words = packed_words(n, ol, cap)
    # pack: GPU per rank vs CPU per rank; the side-entry order differs (atomics), the unpacked rows must not
    pk_cpu = torch.cat([pack_obs(cur[r * n:(r + 1) * n], reset[r * n:(r + 1) * n], cap) for r in range(world)])
    pk_gpu = torch.empty(world * words, dtype=torch.int32, device=gpu)
    for r in range(world):
        view = pk_gpu[r * words:(r + 1) * words]
        view[:1].zero_()
        pack_obs(cur[r * n:(r + 1) * n].to(gpu), reset[r * n:(r + 1) * n].to(gpu), cap, out=view)
    g = pk_gpu.cpu().view(world, words)
    c = pk_cpu.view(world, words)
    side = 4 + n * ol + (n + 31) // 32
    assert torch.equal(g[:, :side], c[:, :side]), "header, o_k rows and bitmap are deterministic"
    out_c = torch.full_like(prev, -1.0)
    age_c = age.clone()
    ovf_c = torch.zeros(1, dtype=torch.int32)
    pred_c = torch.ones(2, world, dtype=torch.int32)
    pred_c[0].zero_()
    unpack_obs(pk_cpu, world, n, ol, cap, a_k, a_p, age_c, prev, out_c, ovf_c, 4, pred_c[0], pred_c[1])
    out_g = torch.full_like(prev, -1.0).to(gpu)
    age_g = age.to(torch.int16).to(gpu)                    # uint16 storage on the GPU
    ovf_g = torch.zeros(1, dtype=torch.int32, device=gpu)
    pred_g = torch.ones(2, world, dtype=torch.int32, device=gpu)
    pred_g[0].zero_()
    unpack_obs(pk_gpu, world, n, ol, cap, a_k.to(gpu), a_p.to(gpu), age_g, prev.to(gpu), out_g, ovf_g, 4, pred_g[0],
               pred_g[1])
    torch.cuda.synchronize()
    same = (out_g.cpu() == out_c) | (torch.isnan(out_g.cpu()) & torch.isnan(out_c))
    assert bool(same.all())
    assert torch.equal(age_g.cpu().to(torch.int32) & 0xFFFF, age_c)
    assert int(ovf_g.item()) == int(ovf_c.item())
    assert torch.equal(pred_g.cpu(), pred_c) and int(pred_c[0].sum()) > 0 and int(pred_c[1].sum()) == 0
    if cap == 10:
        assert int(ovf_g.item()) > 0


def _run_env(rank, world, port, out, backend, n, T, exchange="native"):
    sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))
    os.environ["CF2SIM_EXCHANGE"] = "native" if exchange == "native_env" else exchange
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather, gather_rows
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
    # every env still flying at env-step 41 times out at once: the look-ahead sizes that step's capacity
    pipe = PipelinedObsGather(n, env.obs_dim, dev, delta=True, max_steps=41)
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    acts = torch.rand(T, N, 4, device=dev, generator=g) * 2 - 1      # every rank holds every action
    slab = pipe.start(obs0)
    pipe.drain()
    bad, resets = [], 0
    full = gather_rows(obs0, sizes=[n] * world)
    if not torch.equal(slab, full):
        bad.append(-1)
    for k in range(T):
        a = acts[k]
        a_prev = acts[k - 1] if k > 0 else a
        if exchange == "native_env":       # env-step + exchange in one C call
            j = pipe.k % pipe.depth
            slab = pipe.step_and_publish(env, a[rank * n:(rank + 1) * n].data_ptr(), a.data_ptr(), a_prev.data_ptr())
            pipe.drain()
            ref_obs, ref_done = pipe.obs[j].clone(), pipe.done[j].clone()
        else:
            buf = pipe.buffer()
            done = pipe.done_buffer()
            env.step_raw(a[rank * n:(rank + 1) * n].data_ptr(), obs_ptr=buf.data_ptr(), done_ptr=done.data_ptr())
            ref_obs = buf.clone()
            ref_done = done.clone()
            slab = pipe.publish(a, a_prev)
            pipe.drain()
        full = gather_rows(ref_obs, sizes=[n] * world)
        resets += int(gather_rows(ref_done, sizes=[n] * world).sum())
        if not torch.equal(slab, full):
            bad.append(k)
    torch.cuda.synchronize()
    how = pipe.exchange
    pipe.close()
    if rank == 0:
        with open(out, "w") as f:
            f.write(f"{len(bad)} {resets} {pipe.overflows()} {how} {bad[:3]}")
    dist.destroy_process_group()


def _check(out, T, how):
    nbad, resets, ovf, got = open(out).read().split()[:4]
    assert int(nbad) == 0, open(out).read()
    assert int(resets) > 0 and int(ovf) == 0
    assert got == how


def test_delta_exchange_one_rccl_rank(gpu, tmp_path):
    """The native exchange (cf2_xchg_step: pack, our own RCCL communicator's all-gather, rebuild)."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 32768, 240), nprocs=1, join=True)
    _check(out, 240, "native")


def test_delta_exchange_one_rccl_rank_env_step_in_one_call(gpu, tmp_path):
    """The native exchange's registered form: env-step + exchange per cf2_xchg_env_step call."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 32768, 240, "native_env"), nprocs=1, join=True)
    _check(out, 240, "native")


def test_delta_exchange_one_rccl_rank_torch_path(gpu, tmp_path):
    """The same exchange with the process group's all-gather between the launches from Python."""
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(1, _port(), out, "nccl", 32768, 240, "torch"), nprocs=1, join=True)
    _check(out, 240, "torch")


def test_delta_exchange_two_gloo_ranks_on_one_gpu(gpu, tmp_path):
    out = str(tmp_path / "r.txt")
    mp.spawn(_run_env, args=(2, _port(), out, "gloo", 4096, 240), nprocs=2, join=True)
    _check(out, 240, "gloo")


def test_unpack_rejects_operands_the_kernel_would_overrun(gpu):
    """Host-side checks before the launch: a uint8 age vector (half the bytes the kernel indexes),
    a short slab or a short packed buffer raise ValueError instead of faulting on the device."""
    from cf2sim.dist import pack_obs, packed_words, unpack_obs
    n, ol, cap = 256, 13, 16
    od = 2 * (ol + 4)
    prev = torch.zeros(n, od, device=gpu)
    cur = torch.empty_like(prev)
    a = torch.zeros(n, 4, device=gpu)
    pk = pack_obs(prev, torch.zeros(n, dtype=torch.uint8, device=gpu), cap)
    good_age = torch.zeros(n, dtype=torch.int16, device=gpu)
    unpack_obs(pk, 1, n, ol, cap, a, a, good_age, prev, cur)
    torch.cuda.synchronize()
    with pytest.raises(ValueError):
        unpack_obs(pk, 1, n, ol, cap, a, a, torch.zeros(n, dtype=torch.uint8, device=gpu), prev, cur)
    with pytest.raises(ValueError):
        unpack_obs(pk, 1, n, ol, cap, a, a, good_age, prev, cur[: n // 2])
    with pytest.raises(ValueError):
        unpack_obs(pk[: packed_words(n, ol, cap) // 2], 1, n, ol, cap, a, a, good_age, prev, cur)
    with pytest.raises(ValueError):
        pack_obs(prev, torch.zeros(n, dtype=torch.uint8, device=gpu), cap, out=torch.zeros(8, dtype=torch.int32, device=gpu))
