"""bench.py's launcher contract (no GPU): ``--gpus N`` without torchrun spawns
N rank processes that rendezvous on 127.0.0.1 and only rank 0 prints the JSON
line; a WORLD_SIZE that disagrees with --gpus is refused."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=240)


@pytest.mark.parametrize("n", [2, 3])
def test_spawn_yields_n_ranks_one_json_line(n):
    r = _run(["--gpus", str(n), "--spawn-selftest"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n
    assert d["value"] == n                      # every rank joined the all-reduce
    assert d["rank_sum"] == n * (n - 1) / 2
    assert d["scaling"] == "strong"
    assert d["trajectories_per_step_per_gpu"] == 1024 // n


def test_nested_job_from_ranks():
    """The plumbing of the 8-GPU line's C5 sub-run (bench.run_child_ranks):
    every rank starts one child, the children form their own group on a port
    rank 0 broadcast, and rank 0 attaches the nested job's JSON line."""
    r = _run(["--gpus", "2", "--spawn-selftest", "--selftest-nested"])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] == 2
    assert d["nested"]["n_gpus"] == 2 and d["nested"]["value"] == 2
    assert d["nested"]["rank_sum"] == 1


def test_nested_job_under_torchrun():
    """The driver launches N>1 under torch.distributed.run: the nested job must
    host its own rendezvous (torchrun's agent-store variables are dropped)."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    port = str(29000 + os.getpid() % 1000)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        port, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--spawn-selftest",
                        "--selftest-nested"], env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["nested"]["n_gpus"] == 2 and d["nested"]["value"] == 2


def test_nested_job_hang_is_contained():
    """A nested rank that never finishes is killed at the timeout; the outer
    job still prints its line, with the nested job's error."""
    r = _run(["--gpus", "2", "--spawn-selftest", "--selftest-nested", "--nested-timeout", "20"],
             {"BENCH_SELFTEST_NESTED_HANG_RANK": "1"})
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip().startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] == 2
    assert "error" in d["nested"]


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "8", "--spawn-selftest"], {"WORLD_SIZE": "2", "RANK": "0",
                                                   "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE" in (r.stderr + r.stdout)


def test_failed_rank_ends_the_job():
    """Rank 1 exits before the rendezvous: the parent stops rank 0 (which
    would wait for it forever) and returns rank 1's code."""
    r = _run(["--gpus", "2", "--spawn-selftest"], {"BENCH_SELFTEST_FAIL_RANK": "1"})
    assert r.returncode == 3
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
