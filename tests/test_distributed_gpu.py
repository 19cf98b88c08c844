"""Multi-rank path of the product on a GPU box: two ranks (gloo, both on
cuda:0, as bench.py's CF2_BENCH_BACKEND=gloo rehearsal) each step their contiguous global-id
shard of BatchedCrazyflieEnv; the gathered observations, rewards and dones are bit-identical to
one process stepping all envs, and gather_observations() reassembles the full obs slab (one size
exchange per layout, none per step).  The reference's MPI layer (utils/mpi_tools.py:30-44) plays
the role this replaces for the learner; the env itself needs no collective."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ENV_ID = "DroneHoverBulletFreeEnvWithGust-v0"
T, SEED = 30, 11


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _actions(t, n):
    rng = np.random.default_rng(1000 + t)
    return rng.uniform(-1, 1, size=(n, 4)).astype(np.float32)   # crashes: auto-resets in the window


def _worker(rank, world, port, out_dir, n_total):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "disturbance-crazyfile-simulation_amd"))
    import torch.distributed as dist
    from cf2sim.dist import gather_rows, shard_range
    from cf2sim.vec_env import BatchedCrazyflieEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    off, cnt = shard_range(n_total, rank, world)
    env = BatchedCrazyflieEnv(ENV_ID, cnt, seed=SEED, env_id_offset=off, device="cuda:0")
    env.reset()
    obs = [env.gather_observations().cpu()]
    rew, done = [], []
    kept = []
    for t in range(T):
        a = torch.from_numpy(_actions(t, n_total)[off:off + cnt]).cuda()
        o, r, d, _ = env.step(a)
        gobs = env.gather_observations()
        kept.append(gobs)                       # fresh tensor per call: earlier results stay intact
        obs.append(gobs.cpu())
        rew.append(gather_rows(r).cpu())
        done.append(gather_rows(d).cpu())
    for t in range(T):
        assert torch.equal(kept[t].cpu(), obs[t + 1]), "gather_observations aliased an earlier result"
    assert not torch.equal(kept[0], kept[-1])
    buf = torch.empty_like(kept[0])
    assert env.gather_observations(out=buf) is buf         # opt-in reuse
    env.close()
    if rank == 0:
        np.savez(os.path.join(out_dir, "dist.npz"), obs=torch.stack(obs).numpy(), rew=torch.stack(rew).numpy(),
                 done=torch.stack(done).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_total", [512, 301])     # equal shards / ragged shards
def test_two_ranks_on_gpu_match_one_process(gpu, tmp_path, n_total):
    from cf2sim.vec_env import BatchedCrazyflieEnv
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), n_total), nprocs=2, join=True)
    got = np.load(tmp_path / "dist.npz")
    env = BatchedCrazyflieEnv(ENV_ID, n_total, seed=SEED, device="cuda:0")
    obs = [env.reset().cpu().numpy().copy()]
    rew, done = [], []
    for t in range(T):
        o, r, d, _ = env.step(torch.from_numpy(_actions(t, n_total)).cuda())
        obs.append(o.cpu().numpy().copy())
        rew.append(r.cpu().numpy().copy())
        done.append(d.cpu().numpy().copy())
    env.close()
    np.testing.assert_array_equal(got["obs"], np.stack(obs))
    np.testing.assert_array_equal(got["rew"], np.stack(rew))
    np.testing.assert_array_equal(got["done"], np.stack(done))
    assert np.stack(done).any()          # auto-resets happened inside the compared window
