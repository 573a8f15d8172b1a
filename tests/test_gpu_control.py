"""Adaptive-g runs on the engine vs the reference's committed outputs.

The reference's realtime runs record the g history they used and the
1024-shot forward/echo estimates at each t.  Running the engine's sweep with
that per-period g list (t+1 periods at time t, echo walking the g values back;
controlled-g.py:196-241) must reproduce those estimates within shot noise
(chi^2/dof < 2, |z| < 4.5) — this pins the per-period-g and t_offset=1
semantics on the reference's own adaptive data (L=4 feedback runs, L=20
optimisation run).  Plus an end-to-end CLI run of both scripts."""
import json
import os

import numpy as np
import pytest

from tests.conftest import GOLDEN
from tests.helpers import chi2_per_dof, shot_sigma

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["L4_realtime_gain0.01", "L4_realtime_gain0.05",
                                  "L20_optimization"])
def test_engine_at_reference_g_history(pkg, engine, golden, name):
    with open(os.path.join(GOLDEN, "adaptive.json")) as f:
        case = {c["name"]: c for c in json.load(f)}[name]
    L = case["config"]["L"]
    d = golden["disorder"][f"L{L}"]
    hs, phis = np.array(d["hs"][:1]), np.array(d["phis"][:1])
    g = case["g"]
    T = len(g)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=list(g), noise_prob=0.05, t_offset=1)
    n = 8192 if L == 4 else 2048
    out = engine.autocorr(spec, n, seed=0xC0117)
    for key, ref in (("fwd", case["fwd"]), ("echo", case["echo"])):
        a = out[key][0]
        mine = a.mean(axis=0)
        chi2, zmax = chi2_per_dof(np.array(ref), mine, shot_sigma(mine),
                                  a.std(axis=0) / np.sqrt(n))
        assert chi2 < 2.0 and zmax < 4.5, (name, key, chi2, zmax)


@pytest.mark.parametrize("script,extra", [
    ("controlled-g", ["--exponential_feedback", "0"]),
    ("g-optimization", ["--use_optimization", "1"]),
])
def test_control_cli(pkg, golden, tmp_path, script, extra):
    import pandas as pd

    d = golden["disorder"]["L4"]
    dis = tmp_path / "dis"
    dis.mkdir()
    pd.DataFrame(d["hs"]).to_csv(dis / "hs_L4.csv", index=False)
    pd.DataFrame(d["phis"]).to_csv(dis / "phis_L4.csv", index=False)
    out = tmp_path / "out"
    rc = pkg.control_cli.main(["--script", script, "--L", "4", "--inst", "1", "--tf", "6",
                               "--shots", "256", "--disorder_folder", str(dis),
                               "--out_dir", str(out)] + extra)
    assert rc == 0
    files = sorted(os.listdir(out / "controlled-autocorr_data_L4"))
    assert len(files) == 2
    main = pd.read_csv(out / "controlled-autocorr_data_L4" / files[0])
    assert len(main) == 6 and main["g_history_inst1"][0] == 0.84


def test_control_cli_use_fakebackend(pkg, golden, tmp_path):
    """--use_fakebackend 1 (ctrlg.py:246-250 on FakeBrisbane): device-like noise
    from the stand-in calibration drives the realtime loop and the fixed-g
    comparisons; same folder and files."""
    import pandas as pd

    d = golden["disorder"]["L4"]
    dis = tmp_path / "dis"
    dis.mkdir()
    pd.DataFrame(d["hs"]).to_csv(dis / "hs_L4.csv", index=False)
    pd.DataFrame(d["phis"]).to_csv(dis / "phis_L4.csv", index=False)
    out = tmp_path / "out"
    rc = pkg.control_cli.main(["--L", "4", "--inst", "1", "--tf", "5", "--shots", "256",
                               "--use_fakebackend", "1", "--disorder_folder", str(dis),
                               "--out_dir", str(out)])
    assert rc == 0
    files = sorted(os.listdir(out / "controlled-autocorr_data_L4"))
    assert len(files) == 2
    main = pd.read_csv(out / "controlled-autocorr_data_L4" / files[0])
    assert len(main) == 5 and main["g_history_inst1"][0] == 0.84
    assert np.all(np.abs(main["av_autocorr_echo_adaptive"]) <= 1.0)
