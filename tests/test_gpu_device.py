"""Device-like noise on the HIP engine (dtc_autocorr_device) vs the C oracle.

Same RNG contract on both sides (Philox word 0: Pauli, word 1: amplitude-
damping jump), so every importance-weighted trajectory is the same random
non-unitary circuit: per-trajectory values agree to 1e-10.  The engine's
trajectory means are also checked against the exact density matrix (L=4).
Parity with the reference's FakeBrisbane runs is unpinned (calibration data
unavailable offline).
"""
import os

import numpy as np
import pytest

from oracle import c_oracle, dm_oracle
from tests.helpers import random_disorder

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def harsh_device(pkg, L):
    return pkg.DeviceNoise(p_gate=np.full(L, 0.02), t1_us=np.linspace(1.5, 3.0, L),
                           t2_us=np.linspace(1.0, 4.0, L), gate_ns=120.0, anc_factor=0.9,
                           readout_p01=0.02, readout_p10=0.035)


@pytest.mark.parametrize("L,T,n_traj,state,pol,toff", [
    (4, 10, 6, "vacuum", "x", 0),
    (6, 8, 4, "neel", "xy", 0),
    (12, 7, 3, "vacuum", "y", 1),
    (14, 6, 3, "neel", "circular_left", 0),
    (20, 5, 2, "vacuum", "x", 0),
])
def test_device_engine_matches_oracle(pkg, engine, L, T, n_traj, state, pol, toff):
    rng = np.random.default_rng(L * 7 + T)
    hs, phis = random_disorder(rng, L, 2 if L < 12 else 1)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, polarization=pol,
                         initial_state=state, t_offset=toff, device=harsh_device(pkg, L))
    got = engine.autocorr(spec, n_traj, seed=21, want_zsite=True)
    ref = c_oracle.autocorr(spec, n_traj, seed=21, want_zsite=True)
    for k in ref:
        err = float(np.abs(got[k] - ref[k]).max())
        assert err < 1e-10, (k, err)


def test_device_standin_L20_matches_oracle(pkg, engine, golden):
    cal = pkg.DeviceCalibration.from_json(os.path.join(ROOT, "data", "device_standin_L20.json"))
    d = golden["disorder"]["L20"]
    spec = pkg.SweepSpec(L=20, T=4, hs=np.array(d["hs"])[:1], phis=np.array(d["phis"])[:1],
                         g=0.97, device=cal.device_noise(20))
    got = engine.autocorr(spec, 2, seed=5)
    ref = c_oracle.autocorr(spec, 2, seed=5)
    for k in ref:
        assert float(np.abs(got[k] - ref[k]).max()) < 1e-10


def test_device_batch_invariance(pkg, engine):
    rng = np.random.default_rng(2)
    hs, phis = random_disorder(rng, 13)
    spec = pkg.SweepSpec(L=13, T=5, hs=hs, phis=phis, device=harsh_device(pkg, 13))
    a = engine.autocorr(spec, 6, seed=3, batch=6)
    b = engine.autocorr(spec, 6, seed=3, batch=2)
    for k in a:
        assert np.array_equal(a[k], b[k])


def test_device_means_match_exact_dm(pkg, engine):
    rng = np.random.default_rng(11)
    L, T = 4, 6
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.9, device=harsh_device(pkg, L))
    fe, ee = dm_oracle.device_folded_sweep(L, T, spec.hs[0], spec.phis[0], spec.kick,
                                           spec.device)
    n = 8192
    out = engine.autocorr(spec, n, seed=123)
    for key, exact in (("fwd", fe), ("echo", ee)):
        a = out[key][0]
        se = a.std(axis=0, ddof=1) / np.sqrt(n) + 1e-12
        z = (a.mean(axis=0) - exact) / se
        assert np.max(np.abs(z)) < 4.5, (key, z)


def test_cli_use_fakebackend(pkg, golden, tmp_path):
    """dtc_autocorr.py --use_fakebackend 1: device-like noise from the stand-in
    calibration, fast.py's folder/file names (fakebackend1)."""
    import pandas as pd

    d = golden["disorder"]["L4"]
    dis = tmp_path / "dis"
    dis.mkdir()
    pd.DataFrame(d["hs"]).to_csv(dis / "hs_L4.csv", index=False)
    pd.DataFrame(d["phis"]).to_csv(dis / "phis_L4.csv", index=False)
    out = tmp_path / "out"
    rc = pkg.cli.main(["--L", "4", "--tf", "5", "--use_fakebackend", "1", "--shots", "0",
                       "--trajectories", "64", "--disorder_folder", str(dis),
                       "--out_dir", str(out)])
    assert rc == 0
    files = list((out / "autocorr_data_L4_noiseprob0.05_fakebackend1").glob("autocorr_data_*.csv"))
    assert len(files) == 1
    df = pd.read_csv(files[0])
    assert list(df.columns) == ["time", "av_autocorr", "av_autocorr_echo", "sqrt_av_autocorr_echo"]
    # t = 0: no kicks -> read-out of anc_factor * 1
    cal = pkg.DeviceCalibration.from_json(os.path.join(ROOT, "data", "device_standin_L20.json"))
    dev = cal.device_noise(4)
    assert df["av_autocorr"][0] == pytest.approx(dev.readout(dev.anc_factor), abs=1e-12)


def test_aer_facade_from_backend(pkg):
    """NoiseModel.from_backend(FakeDevice(...)) -> AerSimulator.run(...) (fast.py:77-79,
    152-156, 211-212 with a calibration file instead of FakeBrisbane)."""
    backend = pkg.aer.FakeDevice(os.path.join(ROOT, "data", "device_standin_L20.json"))
    nm = pkg.NoiseModel.from_backend(backend)
    circ = pkg.circuit.dtc_circuit(4, 0, np.zeros(4), np.zeros(3),
                                   lambda step: [[("rx", np.pi * 0.97)] for _ in range(4)])
    sim = pkg.AerSimulator(noise_model=nm, device="GPU", seed_simulator=1)
    counts = sim.run(circ, shots=1000).result().get_counts()
    dev = backend.calibration.device_noise(4)
    a = dev.readout(dev.anc_factor)
    n0 = counts.get("0", 0)
    assert abs(n0 / 1000 - (1 + a) / 2) < 5 * np.sqrt(0.25 / 1000)
    with pytest.raises(NotImplementedError):
        pkg.NoiseModel.from_backend(object())


def test_device_error_paths(pkg, engine):
    rng = np.random.default_rng(0)
    hs, phis = random_disorder(rng, 6)
    bad_p = pkg.DeviceNoise(p_gate=np.full(6, 2.0), t1_us=np.full(6, 100.0),
                            t2_us=np.full(6, 100.0), gate_ns=60.0)
    spec = pkg.SweepSpec(L=6, T=3, hs=hs, phis=phis, device=bad_p)
    with pytest.raises(pkg._capi.DtcError, match="p_gate"):
        engine.autocorr(spec, 2)
    bad_ro = pkg.DeviceNoise(p_gate=np.full(6, 0.01), t1_us=np.full(6, 100.0),
                             t2_us=np.full(6, 100.0), gate_ns=60.0, readout_p01=1.5)
    with pytest.raises(pkg._capi.DtcError, match="read-out"):
        engine.autocorr(pkg.SweepSpec(L=6, T=3, hs=hs, phis=phis, device=bad_ro), 2)
    wrong_L = pkg.DeviceNoise(p_gate=np.full(5, 0.01), t1_us=np.full(5, 100.0),
                              t2_us=np.full(5, 100.0), gate_ns=60.0)
    with pytest.raises(ValueError):
        engine.autocorr(pkg.SweepSpec(L=6, T=3, hs=hs, phis=phis, device=wrong_L), 2)


def test_device_infinite_t1_is_pauli_noise(pkg, engine):
    """T1 = T2 = inf: the device channel is depolarizing only; with anc_factor
    (1-p)^6 and no read-out error it equals dtc_autocorr's exact mean (DM)."""
    rng = np.random.default_rng(4)
    L, T, p = 4, 6, 0.05
    hs, phis = random_disorder(rng, L)
    dev = pkg.DeviceNoise(p_gate=np.full(L, p), t1_us=np.zeros(L), t2_us=np.zeros(L),
                          gate_ns=120.0, anc_factor=(1 - p) ** 6)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, device=dev)
    fe, ee = dm_oracle.folded_sweep(L, T, spec.hs[0], spec.phis[0], spec.kick, p)
    out = engine.autocorr(spec, 4096, seed=17)
    for key, exact in (("fwd", fe), ("echo", ee)):
        a = out[key][0]
        z = (a.mean(axis=0) - exact) / (a.std(axis=0, ddof=1) / np.sqrt(4096) + 1e-12)
        assert np.max(np.abs(z)) < 4.5, (key, z)


# ---- energy path under device-like noise (dtc_energy_device) --------------------

@pytest.mark.parametrize("L,T,n_traj,state,pol", [
    (5, 6, 4, "neel", "x"),
    (7, 5, 3, "vacuum", "xy"),
    (13, 4, 2, "neel", "y"),
    (20, 3, 2, "vacuum", "x"),
])
def test_device_energy_matches_oracle(pkg, engine, L, T, n_traj, state, pol):
    from oracle import energy_oracle

    rng = np.random.default_rng(L + 40)
    hs, phis = random_disorder(rng, L)
    spec = pkg.energy.energy_spec(L, T, hs, phis, 0.92, state, polarization=pol,
                                  device=harsh_device(pkg, L))
    got = engine.energy(spec, n_traj, seed=13)
    for tr in range(n_traj):
        z, zz, x = energy_oracle.trajectory_energy(spec, 0, tr, seed=13)
        assert np.abs(got["z"][0, tr] - z).max() < 1e-10
        assert np.abs(got["zz"][0, tr] - zz).max() < 1e-10
        assert np.abs(got["x"][0, tr] - x).max() < 1e-10


def test_device_energy_means_match_exact_dm(pkg, engine):
    rng = np.random.default_rng(5)
    L, T, n = 5, 6, 8192
    hs, phis = random_disorder(rng, L)
    spec = pkg.energy.energy_spec(L, T, hs, phis, 0.95, "neel", device=harsh_device(pkg, L))
    exact = dm_oracle.energy_sweep(L, T, hs[0], phis[0], spec.kick, 0.0, initial_state="neel",
                                   dev=spec.device)
    got = engine.energy(spec, n, seed=77, batch=1000)
    for k, key in enumerate(("z", "zz", "x")):
        v = got[key][0]
        se = v.std(axis=0, ddof=1) / np.sqrt(n) + 1e-12
        z = (v.mean(axis=0) - exact[k]) / se
        assert np.max(np.abs(z)) < 4.5, (key, z)


def test_energy_cli_use_fakebackend(pkg, golden, tmp_path):
    """energy_cli --mode fakebrisbane (energy-fakebrisbane.py, whose
    --use_fakebackend defaults to 1): folder energy-data_L4-fakebrisbane,
    column energy_p_fakebrisbane = <H>(t) with per-site read-out error, not
    divided by L.  Then energy.py with --use_fakebackend 1: every nprob column
    is the device-noise run, divided by L."""
    import pandas as pd

    d = golden["disorder"]["L4"]
    dis = tmp_path / "dis"
    dis.mkdir()
    pd.DataFrame(d["hs"]).to_csv(dis / "hs_L4.csv", index=False)
    pd.DataFrame(d["phis"]).to_csv(dis / "phis_L4.csv", index=False)
    out = tmp_path / "out"
    rc = pkg.energy_cli.main(["--mode", "fakebrisbane", "--L", "4", "--tf", "4",
                              "--trajectories", "32", "--disorder_folder", str(dis),
                              "--out_dir", str(out)])
    assert rc == 0
    files = list((out / "energy-data_L4-fakebrisbane").glob("energy_data_*.csv"))
    assert len(files) == 1
    df = pd.read_csv(files[0])
    assert list(df.columns) == ["time", "energy_p_fakebrisbane"]
    # t = 0: the vacuum |0000> read out with the per-site flips
    cal = pkg.DeviceCalibration.from_json(os.path.join(ROOT, "data", "device_standin_L20.json"))
    p01, p10 = cal.site_readout(4)
    obs = {"z": np.ones(4), "zz": np.ones(3), "x": np.zeros(4)}
    ro = pkg.energy.readout_observables(obs, p01, p10)
    hs = np.array(d["hs"])[0, :4]
    phis = np.array(d["phis"])[0, :3]
    e0 = pkg.energy.energy_from_observables(ro, 4, 0.97, hs, phis, "full")
    assert df["energy_p_fakebrisbane"][0] == pytest.approx(float(e0), abs=1e-12)
    rc = pkg.energy_cli.main(["--mode", "full", "--use_fakebackend", "1", "--L", "4", "--tf", "4",
                              "--trajectories", "32", "--disorder_folder", str(dis),
                              "--out_dir", str(out)])
    assert rc == 0
    full = list((out / "energy-data_L4-full-ham").glob("energy_data_*.csv"))
    df = pd.read_csv(full[0])
    for p in ("0", "0.001", "0.01", "0.1"):
        assert df[f"energy_p_{p}"][0] == pytest.approx(float(e0) / 4, abs=1e-12)


@pytest.mark.parametrize("L,T,state,pol,toff", [
    (4, 7, "vacuum", "x", 0),        # one site group: every chain starts on it
    (14, 6, "neel", "y", 1),
    (20, 5, "vacuum", "x", 0),       # C3's shape: 12 + 8 sites
    (21, 4, "neel", "circular_left", 0),  # general 2x2 kicks (no factored form)
])
def test_device_dual_pass(pkg, monkeypatch, L, T, state, pol, toff):
    """Device-like noise with the dual pass: the forward runs one kick layer
    ahead (one K-D-K pass per period) and every echo chain's first pass folds
    into it -- dtc_kdk_dual forms K'_1 K_p (input) from the pass's tile after
    its pre-kick (Kraus diagonals of both layers applied) and stores it to E,
    so the run-ahead Kraus layer is never undone.  Without the dual pass
    (DTC_NO_DUAL) nothing runs ahead: K-D forward passes, two per period.  Per
    trajectory: the oracle's values (1e-10), the other schedule's to 1e-12,
    and fewer passes, factored or general kicks."""
    rng = np.random.default_rng(L * 3 + T)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, polarization=pol,
                         initial_state=state, t_offset=toff, device=harsh_device(pkg, L))

    def run(no_dual):
        with monkeypatch.context() as m:
            if no_dual:
                m.setenv("DTC_NO_DUAL", "1")
            with pkg.DtcEngine(0) as eng:
                eng.set_profiling(True)
                out = eng.autocorr(spec, 3, seed=29)
                st = eng.kernel_stats()
                cnt = eng.schedule_counts()
        return (out, st[pkg._capi.KERNEL_LO_PASS]["launches"]
                + st[pkg._capi.KERNEL_HI_PASS]["launches"], cnt)

    got, n_dual, cnt = run(False)
    ref, n_single, cnt_ref = run(True)
    want = c_oracle.autocorr(spec, 3, seed=29)
    for k in want:
        assert float(np.abs(got[k] - want[k]).max()) < 1e-10, k
    assert np.abs(got["echo"] - ref["echo"]).max() < 1e-12
    assert np.abs(got["fwd"] - ref["fwd"]).max() < 1e-13
    assert n_dual < n_single
    # the run-ahead schedule was kept (no silent rebuild with K-D forward
    # passes, which would double the forward passes per period) -- except for
    # one site group (L <= 12): its t = 1 chain is a single pass (undo D^* K'_1),
    # nothing to fold it into, and the undo of a Kraus kick cannot run, so such
    # plans take the K-D schedule, its chains folded into dtc_kd_dual
    if L > 12:
        assert cnt["device_kd"] == 0 and cnt["device_runahead"] == 1 and cnt["folded"] > 0, cnt
    else:
        assert cnt["device_kd"] == 1 and cnt["device_runahead"] == 0 and cnt["folded"] > 0, cnt
    assert cnt_ref == {"folded": 0, "device_runahead": 0, "device_kd": 1, "split13": 0}, cnt_ref


@pytest.mark.parametrize("L,T,pol", [(14, 6, "x"), (20, 5, "circular_left")])
def test_device_kd_dual_forced(pkg, monkeypatch, L, T, pol):
    """The K-D schedule under device-like noise, forced (DTC_NO_RUNAHEAD=1: the
    schedule the engine falls back to when an echo chain cannot fold into the
    run-ahead dual pass): the forward closes each period with a K-D pass and
    every chain's first D^* K'_1 pass folds into it (dtc_kd_dual).  Per
    trajectory: the oracle's values (1e-10) and the run-ahead schedule's
    (1e-12), with more forward passes than the run-ahead schedule."""
    rng = np.random.default_rng(L * 5 + T)
    hs, phis = random_disorder(rng, L, 1)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, polarization=pol,
                         initial_state="neel", device=harsh_device(pkg, L))

    def run(forced):
        with monkeypatch.context() as m:
            if forced:
                m.setenv("DTC_NO_RUNAHEAD", "1")
            with pkg.DtcEngine(0) as eng:
                eng.set_profiling(True)
                out = eng.autocorr(spec, 4, seed=31)
                st = eng.kernel_stats()
                cnt = eng.schedule_counts()
        return (out, st[pkg._capi.KERNEL_LO_PASS]["launches"]
                + st[pkg._capi.KERNEL_HI_PASS]["launches"], cnt)

    kd, n_kd, cnt_kd = run(True)
    ahead, n_ahead, cnt_ahead = run(False)
    want = c_oracle.autocorr(spec, 4, seed=31)
    for k in want:
        assert float(np.abs(kd[k] - want[k]).max()) < 1e-10, k
        assert float(np.abs(kd[k] - ahead[k]).max()) < 1e-12, k
    assert cnt_kd["device_kd"] == 1 and cnt_kd["device_runahead"] == 0, cnt_kd
    assert cnt_kd["folded"] > 0, cnt_kd  # the K-D dual pass ran
    assert cnt_ahead["device_kd"] == 0, cnt_ahead
    assert n_kd > n_ahead


def test_device_dual_batches_and_t_first(pkg, engine):
    """The device dual pass under the schedule's other shapes: two instances,
    batches that split the octets (batch invariance is exact), echo-only and
    t_first > 0 runs (the chains at t < t_first are not built, so the fold
    lands on other forward passes), each against the oracle per trajectory."""
    rng = np.random.default_rng(41)
    hs, phis = random_disorder(rng, 16, 2)
    spec = pkg.SweepSpec(L=16, T=6, hs=hs, phis=phis, g=0.91, polarization="x",
                         initial_state="neel", device=harsh_device(pkg, 16))
    a = engine.autocorr(spec, 10, seed=13, batch=20)
    b = engine.autocorr(spec, 10, seed=13, batch=3)
    for k in a:
        assert np.array_equal(a[k], b[k]), k
    ref = c_oracle.autocorr(spec, 10, seed=13)
    for k in ref:
        assert float(np.abs(a[k] - ref[k]).max()) < 1e-10, k
    e = engine.autocorr(spec, 10, seed=13, want_fwd=False)
    assert np.abs(e["echo"] - ref["echo"]).max() < 1e-10
    late = engine.autocorr(spec, 10, seed=13, t_first=3)
    ref_late = c_oracle.autocorr(spec, 10, seed=13, t_first=3)
    for k in ref_late:
        assert float(np.abs(late[k] - ref_late[k]).max()) < 1e-10, k
        assert np.abs(late[k][..., 3:] - a[k][..., 3:]).max() < 1e-12, k
