"""bench.py --gpus 2 end to end on a one-GPU box: the launcher spawns two rank
processes, each drives the HIP engine and joins the final all-reduce, and only
rank 0 prints the JSON line.  BENCH_SHARE_DEVICE=1 puts both ranks on GPU 0
with gloo collectives (RCCL refuses two ranks on one GPU), so this checks the
multi-rank plumbing the driver's 8-GPU run uses, not its scaling."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["BENCH_SHARE_DEVICE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_c2_two_spawned_ranks():
    d = _run(["--gpus", "2", "--steps", "1", "--warmup", "0", "--strong-total", "64",
              "--no-cpu-baseline"])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["trajectories_per_step"] == 64
    assert d["config"]["trajectories_per_step_per_gpu"] == 32
    assert len(d["roofline"]["per_rank_GBps"]) == 2
    assert all(x and x > 0 for x in d["roofline"]["per_rank_GBps"])
    # t = 0 of the all-reduced autocorrelator: (1-p)^6 exactly, forward and echo
    assert abs(d["autocorr_t0_3"]["fwd"][0] - 0.95 ** 6) < 1e-12
    assert abs(d["autocorr_t0_3"]["echo"][0] - 0.95 ** 6) < 1e-12
    assert d["value"] > 0


def test_c4_two_spawned_ranks():
    d = _run(["--config", "c4", "--gpus", "2", "--steps", "1", "--warmup", "0",
              "--instances", "2", "--tf", "4"])
    assert d["n_gpus"] == 2
    assert abs(d["z_mean_t1"] - __import__("math").cos(__import__("math").pi * 0.97)) < 1e-12
