"""Adaptive-g controllers and envelopes (no GPU).

* controller updates reproduce the reference's own g histories bit-for-bit
  (autocorr_data_L4 realtime runs: linear feedback, g_max 1.0 and 0.95);
* find_envelope reproduces every envelope column the reference committed
  (polarization and controlled-g variants);
* the realtime loop / optimiser / CSV writer run end to end with the C oracle
  standing in for the engine (small L), and the CSV columns equal the
  reference's controlled-autocorr_data_L20 header.
"""
import json
import os

import numpy as np
import pytest

from oracle import c_oracle
from tests.conftest import GOLDEN


def _adaptive():
    with open(os.path.join(GOLDEN, "adaptive.json")) as f:
        return {c["name"]: c for c in json.load(f)}


@pytest.mark.parametrize("name,g_max", [("L4_realtime_gain0.01", 1.0),
                                        ("L4_realtime_gain0.05", 0.95)])
def test_linear_feedback_reproduces_reference_history(pkg, name, g_max):
    c = _adaptive()[name]
    cfg = pkg.control.ControllerConfig(feedback_gain=c["config"]["gain"], exponential_feedback=0,
                                       g_min=0.84, g_max=g_max)
    g, e = c["g"], c["echo"]
    pred = [pkg.control.feedback_update(e[t], g[t], t, cfg) for t in range(len(g) - 1)]
    assert np.abs(np.array(pred) - np.array(g[1:])).max() < 1e-15


def test_exponential_feedback_rule(pkg):
    cfg = pkg.control.ControllerConfig(feedback_gain=0.02, decay_compensation=0.1, g_max=1.0)
    for echo, g, t in ((0.6, 0.85, 0), (0.3, 0.9, 5), (0.005, 0.9, 3), (1.2, 0.9, 2)):
        err = 1.0 - echo
        log_term = (0.02 * np.log(1.0 / echo) * 0.1 if 0.01 < echo < 1.0 else
                    (0.0 if echo >= 1.0 else 0.04))
        want = np.clip(g + (0.02 * err * np.exp(0.1 * t) + log_term) * (1 + 0.1 * t), 0.84, 1.0)
        assert abs(pkg.control.feedback_update(echo, g, t, cfg) - want) < 1e-15


def test_batch_adjust(pkg):
    cfg = pkg.control.ControllerConfig(feedback_gain=0.1, g_min=0.8, g_max=0.9)
    out = pkg.control.adjust_g_based_on_echo([0.5, 0.2, 0.9], [0.84, 0.84, 0.84], cfg)
    assert out == [0.84, 0.89, 0.9]


def test_envelopes_match_reference(pkg):
    with open(os.path.join(GOLDEN, "envelopes.json")) as f:
        cases = json.load(f)
    assert len(cases) >= 30
    for c in cases:
        up, lo = pkg.envelopes.find_envelope(np.array(c["signal"], float), c["window"],
                                             c["variant"])
        np.testing.assert_allclose(up, np.array(c["upper"], float), rtol=0, atol=1e-12,
                                   equal_nan=True)
        np.testing.assert_allclose(lo, np.array(c["lower"], float), rtol=0, atol=1e-12,
                                   equal_nan=True)


def test_envelope_controlled_variant_needs_four_extrema(pkg):
    with pytest.raises(pkg.envelopes.EnvelopeUnavailable):
        pkg.envelopes.find_envelope(np.array([0.0, 1.0, 0.5]), 3, "controlled")
    up, lo = pkg.envelopes.find_envelope(np.array([0.0, 1.0, 0.5]), 3, "polarization")
    assert np.all(up >= [0.0, 1.0, 0.5]) and np.all(lo <= [0.0, 1.0, 0.5])


class OracleEngine:
    """The C oracle behind the engine's autocorr signature (CPU stand-in)."""

    def autocorr(self, spec, n_traj, seed=0, traj_offset=0, want_fwd=True, want_echo=True,
                 want_zsite=False, batch=0, t_first=0):
        return c_oracle.autocorr(spec, n_traj, seed=seed, traj_offset=traj_offset,
                                 want_fwd=want_fwd, want_echo=want_echo, want_zsite=want_zsite,
                                 n_threads=4, t_first=t_first)


@pytest.mark.parametrize("opt", [0, 1])
def test_realtime_loop_and_outputs(pkg, golden, tmp_path, opt):
    ct = pkg.control
    d = golden["disorder"]["L4"]
    hs, phis = np.array(d["hs"])[:, :4], np.array(d["phis"])[:, :3]
    cfg = ct.ControllerConfig(feedback_gain=0.05, exponential_feedback=1, g_max=0.95,
                              use_optimization=opt)
    eng = OracleEngine()
    T = 4
    ad = ct.realtime_adaptive(4, T, hs, phis, 0.84, cfg, shots=32, engine=eng)
    assert ad.g.shape == (1, T) and ad.g[0, 0] == 0.84
    assert np.all((ad.g >= 0.84) & (ad.g <= 0.95))
    assert np.all(np.abs(ad.echo) <= 1) and np.all(np.abs(ad.forward) <= 1)
    std84 = ct.fixed_g_sweep(4, T, hs, phis, 0.84, shots=32, engine=eng)
    std97 = ct.fixed_g_sweep(4, T, hs, phis, 0.97, shots=32, engine=eng)
    main, comp = ct.write_controlled_outputs(str(tmp_path), "vacuum", 4, 1, 0.84, cfg, ad,
                                             std84, std97, (1, 0.0, 1.0, 0.05, 1),
                                             optimization_script=bool(opt))
    import pandas as pd

    cols = list(pd.read_csv(main).columns)
    ref_cols = _adaptive()["L20_optimization"]["columns"]
    base = [c for c in ref_cols if "env" not in c]
    assert [c for c in cols if "env" not in c] == base
    if opt:
        assert "optimization_iter5" in os.path.basename(main)
        assert "adaptive_optimization_vs_fixed" in os.path.basename(comp)
    else:
        assert "_exp0.1_" in os.path.basename(main)


def test_realtime_loop_device_noise(pkg, golden):
    """Device-like noise through the controllers (the C oracle as the engine):
    estimates come from shots drawn on the trajectory mean, and the loop's
    first estimate matches the exact density matrix within shot noise."""
    from oracle import dm_oracle

    ct = pkg.control
    d = golden["disorder"]["L4"]
    hs, phis = np.array(d["hs"])[:, :4], np.array(d["phis"])[:, :3]
    dev = pkg.DeviceNoise(p_gate=np.full(4, 0.02), t1_us=np.full(4, 2.0), t2_us=np.full(4, 2.5),
                          gate_ns=120.0, anc_factor=0.9, readout_p01=0.02, readout_p10=0.03)
    cfg = ct.ControllerConfig(feedback_gain=0.05, exponential_feedback=1, g_max=0.95)
    eng = OracleEngine()
    ad = ct.realtime_adaptive(4, 3, hs, phis, 0.84, cfg, shots=2048, engine=eng, device=dev)
    assert ad.g[0, 0] == 0.84 and np.all((ad.g >= 0.84) & (ad.g <= 0.95))
    spec = pkg.SweepSpec(L=4, T=1, hs=hs[:1], phis=phis[:1], g=[0.84], t_offset=1)
    fe, ee = dm_oracle.device_folded_sweep(4, 1, hs[0], phis[0], spec.kick, dev, t_offset=1)
    sd = 1.0 / np.sqrt(2048)
    assert abs(ad.forward[0, 0] - fe[0]) < 5 * sd and abs(ad.echo[0, 0] - ee[0]) < 5 * sd
    f84, e84 = ct.fixed_g_sweep(4, 3, hs, phis, 0.84, shots=256, engine=eng, device=dev)
    assert f84.shape == (1, 3) and np.all(np.abs(e84) <= 1)
