"""bench.py's multi-rank measurement path on a GPU box.

- `bench.py --gpus 2` without a launcher starts its own two ranks (CF2_BENCH_BACKEND=gloo: both
  ranks share the one MI355X of the test box) and prints one line with n_gpus = world_size = 2
  whose value is BASELINE configs[3]: the 262 144 envs split over the ranks with the observation
  all-gather in the timed region ("scaling": "strong"), plus the collective-free split and the
  weak-scaling key.
- Under torchrun with one rank and --gather-obs, the RCCL ("nccl") native exchange runs (batches
  of env-steps with the pack fused in, one all-gather + consume each), the path the 8-GPU run
  takes; its rows equal a full all-gather.
- PipelinedObsGather's output equals the observations the env-step wrote, step for step."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHORT = ["--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--rollout-k", "0", "--streaming-ring", "0",
         "--oc-envs", "0", "--strong-steps", "20", "--weak-steps", "20", "--gather-steps", "40", "--collect-steps", "0",
         "--exchange-probe", "0"]


def _env():
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    return e


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _line(stdout):
    lines = [l for l in stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_bench_self_launches_two_ranks(gpu):
    env = dict(_env(), CF2_BENCH_BACKEND="gloo")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *SHORT], env=env,
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    assert d["n_gpus"] == 2 and d["world_size"] == 2 and d["backend"] == "gloo"
    # the headline is BASELINE configs[3]: the 262 144 envs split over the ranks with the
    # observation all-gather of every env-step inside the timed region (strong scaling)
    assert d["config"]["global_envs"] == 262144 and d["config"]["envs_per_gpu"] == 131072
    assert d["scaling"] == "strong" and d["config"]["gather_obs"] is True and "gather_error" not in d["config"]
    gi = d["gather"]
    assert d["value"] == gi["value"] > 0 and d["ms_per_step"] == gi["ms_per_step"]
    assert gi["global_envs"] == 262144 and gi["steps"] == d["steps"] == 20
    # the delta exchange (default): 2.3x fewer bytes than the rows, no side-slab overflow, the rows
    # on request equal to a full all-gather
    assert gi["mode"].startswith("delta rows") and gi["exchange"] == "gloo" and gi["envs_per_gpu"] == 131072
    assert gi["full_rows_bytes_per_rank_per_step"] == 131072 * 34 * 4
    assert gi["bytes_per_rank_per_step"] * 2.3 <= gi["full_rows_bytes_per_rank_per_step"]
    assert gi["overflows"] == 0 and gi["rows_on_request"]["equal_to_full_gather"] is True
    # the extra keys: the same split without the gather (the fallback headline) and every rank
    # stepping 262 144 envs of its own (weak scaling)
    cf = d["collective_free"]
    assert cf["global_envs"] == 262144 and cf["gather_obs"] is False and cf["value"] > 0
    w = d["weak_scaling"]
    assert w["global_envs"] == 2 * 262144 and w["envs_per_gpu"] == 262144 and w["value"] > 0


def test_bench_two_ranks_native_exchange_headline(gpu):
    """The 8-GPU headline's code path at world size 2 on one GPU: bench.py --gpus 2 over gloo with the
    native exchange bound to the tests' RCCL stand-in (CF2SIM_RCCL_PATH), so the gathered headline
    runs PipelinedObsGather.run's batches (cf2_xchg_run: the [world][nb][words] receive layout,
    both ranks' look-ahead counts) inside the timed region; the rows of the last step equal a full
    all-gather and nothing overflows."""
    standin = os.path.join(ROOT, "tests", "standin_rccl", "_build", "libstandin_rccl.so")
    assert os.path.exists(standin)
    # a batch of 16 packed buffers of 131 072 envs is ~120 MB per rank: the stand-in's slots are sized for it
    env = dict(_env(), CF2_BENCH_BACKEND="gloo", CF2SIM_RCCL_PATH=standin, CF2_STANDIN_SLOT_MB="160")
    args = [a if a != "20" else "48" for a in SHORT]          # three batches of 16 timed env-steps
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *args], env=env,
                       capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    gi = d["gather"]
    assert gi["exchange"] == "native" and "cf2_xchg_run" in gi["launch"], gi
    assert d["config"]["gather_obs"] is True and d["value"] == gi["value"] > 0 and gi["global_envs"] == 262144
    assert gi["steps"] == d["steps"] == 48 and gi["envs_per_gpu"] == 131072
    assert gi["overflows"] == 0 and gi["rows_on_request"]["equal_to_full_gather"] is True


def test_bench_rccl_gather_path_one_rank(gpu):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1", "--gather-obs",
           "--gather-envs", "32768", *SHORT]
    p = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    assert d["backend"] == "nccl" and d["world_size"] == 1 and d["config"]["gather_obs"] is True
    gi = d["gather"]
    assert gi["mode"].startswith("delta rows") and gi["exchange"] == "native" and d["value"] > 0
    assert gi["overflows"] == 0 and gi["rows_on_request"]["equal_to_full_gather"] is True
    assert "cf2_xchg_run" in gi["launch"]


def _pipe_worker(rank, world, port, out):
    sys.path.insert(0, os.path.join(ROOT, "disturbance-crazyfile-simulation_amd"))
    import torch.distributed as dist
    from cf2sim.dist import PipelinedObsGather
    from cf2sim.vec_env import BatchedCrazyflieEnv
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    n = 4096
    env = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=3, device="cuda:0")
    ref = BatchedCrazyflieEnv("DroneHoverBulletFreeEnvWithGust-v0", n, seed=3, device="cuda:0")
    env.reset()
    ref.reset()
    pipe = PipelinedObsGather(n, env.obs_dim, torch.device("cuda", 0), depth=2)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(5)
    outs, refs = [], []
    for k in range(12):
        a = torch.rand(n, 4, device="cuda:0", generator=g) * 2 - 1
        buf = pipe.buffer()
        env.step_raw(a.data_ptr(), obs_ptr=buf.data_ptr())
        o = pipe.publish()
        ref.step(a)
        refs.append(ref.obs.clone())
        if k % 2:
            pipe.drain()
            outs.append((k, o.clone()))
    pipe.drain()
    torch.cuda.synchronize()
    ok = all(torch.equal(o, refs[k]) for k, o in outs)
    with open(out, "w") as f:
        f.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


def test_pipelined_gather_matches_env_obs(gpu, tmp_path):
    import torch.multiprocessing as mp
    out = str(tmp_path / "res.txt")
    mp.spawn(_pipe_worker, args=(1, _port(), out), nprocs=1, join=True)
    assert open(out).read() == "ok"


def test_bench_hj_config_runs_the_node_shard_probe(gpu):
    # every BASELINE config goes through the same line (tools/all_configs.sh): on the HJ-adversary
    # env the node-shard exchange probe's own env must have value tables bound too
    assert SHORT[-2:] == ["--exchange-probe", "0"]
    args = SHORT[:-2] + ["--exchange-probe", "1"]
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--env-id",
                        "DroneHoverBulletFreeEnvWithAdversary-v0", *args], env=_env(), capture_output=True,
                       text=True, timeout=600, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    d = _line(p.stdout)
    assert d["value"] > 0 and "synthetic 15^6 HJ value tables" in d["data"]
    x = d["delta_exchange"]
    assert x["node_shard_step_us"] > 0 and x["node_shard_step_packed_us"] > 0
