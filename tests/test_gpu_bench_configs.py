"""bench.py's other lines end to end on one GPU at small sizes (so the bench
paths the driver and the profiles use cannot rot): energy, C3, C5 (virtual
ranks), the adaptive-g controller, and the C5 sub-run that the 8-GPU line
carries, forced on one GPU.  Each must print one JSON line whose physics
sanity values hold (the C5 known answer <Z_i(1)> = cos(pi g) from vacuum)."""
import json
import math
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COS = math.cos(math.pi * 0.97)


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                       capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_energy_line():
    d = _run(["--config", "energy", "--steps", "1", "--warmup", "0", "--batch", "16",
              "--tf", "5", "--no-cpu-baseline"])
    assert d["value"] > 0 and d["roofline"]["achieved"] > 0
    e = d["energy_per_site_t0_3"]
    assert len(e) == 4 and all(math.isfinite(x) for x in e)


def test_c3_line():
    d = _run(["--config", "c3", "--steps", "1", "--warmup", "0", "--strong-total", "32",
              "--tf", "5", "--no-cpu-baseline"])
    assert d["value"] > 0 and d["config"]["trajectories_per_step"] == 32
    assert all(math.isfinite(x) for x in d["autocorr_t0_3"]["echo"])


def test_c5_virtual_line():
    d = _run(["--config", "c5", "--L", "24", "--tf", "4", "--steps", "1", "--warmup", "0"])
    assert d["config"]["shards"] == 8 and d["config"]["L"] == 24
    assert abs(d["z_t1_mean"] - COS) < 1e-12


def test_ctrl_line():
    d = _run(["--config", "ctrl", "--ctrl-tf", "3", "--steps", "1", "--warmup", "0",
              "--no-cpu-baseline"])
    assert d["value"] > 0 and len(d["g_history_mean"]) == 3
    assert abs(d["g_history_mean"][0] - 0.84) < 1e-12


def test_c5_subrun_forced():
    """The nested C5 job of the 8-GPU line (BENCH_C5_SUBRUN=1 forces it at one
    rank: 8 virtual shards of L=31)."""
    d = _run(["--steps", "1", "--warmup", "0", "--strong-total", "32", "--tf", "4",
              "--no-cpu-baseline"], {"BENCH_C5_SUBRUN": "1"})
    assert "error" not in d["c5"], d["c5"]
    assert d["c5"]["config"]["shards"] == 8
    assert abs(d["c5"]["z_t1_mean"] - COS) < 1e-12
    # (in place on one GPU the exchange is fused into the slice kicks: no window)
    assert d["c5"]["exchange"]["per_period_ms"] > 0 or d["c5"]["exchange"]["fused_into_kick_pass"]
