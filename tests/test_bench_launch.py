"""bench.py's multi-GPU launch on the CPU: the launch plan (one child process per rank, rank r on
local GPU r, rendezvous on 127.0.0.1), that the planned ranks really form one process group
(gloo, world size 2 and 4), that a failing rank fails the launch, and the shard arithmetic of
BASELINE's metric config (262 144 envs over the job, a contiguous global-id shard per rank).
The reference's launcher for this role is mpi_fork (utils/mpi_tools.py:47-99)."""
import json
import os
import socket
import sys

import pytest

import bench
from cf2sim.dist import launch_plan, run_ranks, shard_range

RANK_SCRIPT = r"""
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group("gloo")
t = torch.tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
fail = int(os.environ.get("FAIL_RANK", "-1"))
if dist.get_rank() == fail:
    sys.exit(3)
with open(os.path.join(sys.argv[1], f"rank{dist.get_rank()}.json"), "w") as f:
    json.dump({"rank": dist.get_rank(), "world": dist.get_world_size(), "sum": float(t.item()),
               "local_rank": int(os.environ["LOCAL_RANK"]), "argv": sys.argv[2:]}, f)
dist.barrier()
dist.destroy_process_group()
"""


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_launch_plan_environment():
    plan = launch_plan(4, 29511, "/x/bench.py", ["--gpus", "4", "--steps", "7"], base_env={"KEEP": "1"},
                       python="/usr/bin/python3")
    assert len(plan) == 4
    for r, (cmd, env) in enumerate(plan):
        assert cmd == ["/usr/bin/python3", "-u", "/x/bench.py", "--gpus", "4", "--steps", "7"]
        assert env["RANK"] == env["LOCAL_RANK"] == str(r)
        assert env["WORLD_SIZE"] == env["LOCAL_WORLD_SIZE"] == "4"
        assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29511"
        assert env["KEEP"] == "1"
    with pytest.raises(ValueError):
        launch_plan(0, 1, "x", [])


@pytest.mark.parametrize("world", [2, 4])
def test_planned_ranks_form_one_process_group(tmp_path, world):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    rc = run_ranks(launch_plan(world, _port(), str(script), [str(tmp_path), "--steps", "3"]), timeout=120)
    assert rc == 0
    got = [json.loads((tmp_path / f"rank{r}.json").read_text()) for r in range(world)]
    assert [g["rank"] for g in got] == list(range(world))
    assert all(g["world"] == world and g["local_rank"] == g["rank"] for g in got)
    assert all(g["sum"] == world * (world + 1) / 2 for g in got)
    assert all(g["argv"] == ["--steps", "3"] for g in got)


def test_failing_rank_fails_the_launch(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    env = dict(os.environ, FAIL_RANK="1")
    rc = run_ranks(launch_plan(2, _port(), str(script), [str(tmp_path)], base_env=env), timeout=120)
    assert rc == 3


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_metric_config_shards(world):
    spans = [shard_range(bench.METRIC_GLOBAL_ENVS, r, world) for r in range(world)]
    assert [c for _, c in spans] == [262144 // world] * world
    assert [o for o, _ in spans] == [r * (262144 // world) for r in range(world)]


def test_bench_defaults_are_the_metric_config():
    a = bench.parse_args([])
    # BASELINE configs[3]: 262 144 envs over the whole job, split over the ranks, with the north
    # star's observation all-gather (the headline at N > 1); --scaling weak: 262 144 on every rank
    assert a.scaling == "strong" and a.envs_per_gpu is None and a.gather_envs == 262144
    assert a.global_envs == 262144 and bench.parse_args(["--scaling", "weak"]).scaling == "weak"
    assert a.gather_obs is None          # on at N > 1, off at N = 1
    assert a.steps == 10000 and a.warmup == 1000
    assert bench.parse_args(["--no-gather-obs"]).gather_obs is False


def test_gpus_mismatch_with_launcher_aborts(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "2")
    with pytest.raises(SystemExit, match="launcher started 2 ranks"):
        bench.main(["--gpus", "4"])


def test_self_launch_propagates_rank_failure(tmp_path, monkeypatch):
    """bench.py --gpus 2 without a launcher starts two ranks; a rank that fails (here: malformed
    --env-kw, before any GPU work) makes the parent exit non-zero."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CF2_BENCH_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--env-kw", "not json"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "JSONDecodeError" in p.stderr                  # a child ran and failed


def _line(value=1.0):
    return {"value": value, "steps": 10, "ms_per_step": 0.5, "config": {
        "workload": "w", "parallelism": "env-shard x8, no data-path collective", "gather_obs": False,
        "gather_error": "the gathered run had not completed"}}


def test_gathered_headline_replaces_the_collective_free_value():
    """N > 1: a successful gather is the headline (BASELINE configs[3]: 262 144 envs split over the
    ranks, the observation all-gather in the timed region)."""
    info = {"value": 2e10, "ms_per_step": 0.013, "steps": 10, "exchange": "native",
            "mode": "delta rows (o_k + ...)", "global_envs": 262144}
    line = bench.merge_gather(_line(), info, True, 8, "nccl")
    assert line["value"] == 2e10 and line["ms_per_step"] == 0.013 and line["gather"] is info
    cf = line["config"]
    assert cf["gather_obs"] is True and "gather_error" not in cf and "RCCL all-gather" in cf["parallelism"]


def test_failed_gather_keeps_the_collective_free_split_never_the_weak_figure():
    line = bench.merge_gather(_line(7.0), {"error": "RuntimeError('x')"}, True, 8, "nccl")
    assert line["value"] == 7.0 and line["config"]["gather_obs"] is False
    assert line["config"]["gather_error"] == "RuntimeError('x')"


def test_gather_as_an_extra_key_leaves_the_headline():
    info = {"value": 3.0, "ms_per_step": 1.0, "steps": 40, "exchange": "native", "mode": "delta rows"}
    line = bench.merge_gather(_line(5.0), info, False, 1, "nccl")
    assert line["value"] == 5.0 and line["gather"] is info and line["steps"] == 10
