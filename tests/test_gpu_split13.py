"""The 13 / 7 site split of L = 20 (round 6): a 13-site group in 8192-amplitude
tiles (dtc_tile13.hip) and a 7-site column group (pass_body kGeoB7: tile bits
0..4 = sites 0..4 as 512-B runs, 5..11 = sites 13..19).  L = 20 sweeps run it
with DTC_SPLIT13=1 (unitary factored kicks, probe only, no prefix); the
default keeps the 12 / 8 split (the 13 / 7 one measured slower, round 6).  Per trajectory the two schedules compute the same
quantity (the Floquet period of autocorr-delta-a-single-qiskit-fast.py:111-121
and the echo, :140-147), so they agree to rounding, and both equal the C
oracle to 1e-10."""
import json
import os

import numpy as np
import pytest

from oracle import c_oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _row0(pkg, n=1):
    with open(os.path.join(ROOT, "tests", "golden", "disorder.json")) as f:
        d = json.load(f)["L20"]
    return np.array(d["hs"][:n]), np.array(d["phis"][:n])


def _run(pkg, monkeypatch, spec, n_traj, split, **kw):
    with monkeypatch.context() as m:
        if split:
            m.setenv("DTC_SPLIT13", "1")
        with pkg.DtcEngine(0) as eng:
            out = eng.autocorr(spec, n_traj, **kw)
            cnt = eng.schedule_counts()
            eng.release_buffers()
    return out, cnt


@pytest.mark.parametrize("pol,state,toff,noise,batch", [
    ("x", "vacuum", 0, 0.05, 16),    # the headline's kicks, octet layout
    ("y", "neel", 0, 0.05, 16),      # RY family
    ("x", "neel", 1, 0.03, 3),       # t_offset = 1, contiguous states (batch < 8)
    ("x", "vacuum", 0, 0.0, 8),      # noiseless
])
def test_split13_matches_12_8_and_oracle(pkg, engine, monkeypatch, pol, state, toff, noise, batch):
    engine.release_buffers()
    hs, phis = _row0(pkg)
    T = 9
    spec = pkg.SweepSpec(L=20, T=T, hs=hs, phis=phis, g=0.97, noise_prob=noise,
                         use_noise=1 if noise else 0, polarization=pol, initial_state=state,
                         t_offset=toff)
    n = 16
    s13, c13 = _run(pkg, monkeypatch, spec, n, True, seed=77, traj_offset=5, batch=batch)
    s12, c12 = _run(pkg, monkeypatch, spec, n, False, seed=77, traj_offset=5, batch=batch)
    assert c13["split13"] == (n + batch - 1) // batch and c12["split13"] == 0, (c13, c12)
    for k in ("fwd", "echo"):
        assert np.abs(s13[k] - s12[k]).max() < 1e-12, k
    ids = [0, 7, 15]
    for i in ids:
        ref = c_oracle.autocorr_fused(spec, 1, seed=77, traj_offset=5 + i)
        for k in ("fwd", "echo"):
            err = float(np.abs(s13[k][0, i] - ref[k][0, 0]).max())
            assert err < 1e-10, (k, i, err)


def test_split13_headline_batch_and_t_first(pkg, engine, monkeypatch):
    """The bench line's own schedule (T = 30, B = 1024, dual passes on the
    7-site group, 12-site light-cone ends) with and without the split: equal
    to rounding, and t_first = 20 runs equal to the full run."""
    engine.release_buffers()
    hs, phis = _row0(pkg)
    spec = pkg.SweepSpec(L=20, T=30, hs=hs, phis=phis, g=0.97, noise_prob=0.05, use_noise=1,
                         initial_state="vacuum")
    s13, c13 = _run(pkg, monkeypatch, spec, 1024, True, seed=0x5EED0001, batch=1024)
    s12, _ = _run(pkg, monkeypatch, spec, 1024, False, seed=0x5EED0001, batch=1024)
    assert c13["split13"] == 1 and c13["folded"] > 0, c13
    for k in ("fwd", "echo"):
        assert np.abs(s13[k] - s12[k]).max() < 1e-12, k
    late, _ = _run(pkg, monkeypatch, spec, 64, True, seed=0x5EED0001, batch=64, t_first=20)
    for k in ("fwd", "echo"):
        assert np.abs(late[k][..., 20:] - s13[k][:, :64, 20:]).max() < 1e-13, k
