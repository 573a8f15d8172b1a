"""Device-like noise (use_fakebackend=1 stand-in; include/dtc.h dtc_device_noise), CPU.

Parity with the reference is unpinned (FakeBrisbane's calibration is not
available offline, and no FakeBrisbane output is committed in the reference).
What is pinned here is the model:
1. the exact density matrix of the channel is trace preserving and reduces to
   the depolarizing-only sweep when T1 = T2 = inf;
2. the C oracle's importance-weighted trajectories (fixed jump probability
   gamma/2, weight 1/sqrt(q)) average to the exact density-matrix values;
3. the calibration loader maps the committed stand-in file to per-site
   channels (kick = 2 sx pulses, ancilla factor, read-out).
"""
import os

import numpy as np
import pytest

from oracle import c_oracle, dm_oracle
from tests.helpers import random_disorder

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def harsh_device(pkg, L):
    """Exaggerated noise so that a few thousand trajectories resolve it."""
    return pkg.DeviceNoise(p_gate=np.full(L, 0.02), t1_us=np.linspace(1.5, 3.0, L),
                           t2_us=np.linspace(1.0, 4.0, L), gate_ns=120.0, anc_factor=0.9,
                           readout_p01=0.02, readout_p10=0.035)


def test_channel_reduces_to_depolarizing(pkg):
    rng = np.random.default_rng(3)
    L, T = 4, 5
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.97, noise_prob=0.05)
    dev = pkg.DeviceNoise(p_gate=np.full(L, 0.05), t1_us=np.zeros(L), t2_us=np.zeros(L),
                          gate_ns=100.0, anc_factor=(1 - 0.05) ** 6)
    f0, e0 = dm_oracle.folded_sweep(L, T, spec.hs[0], spec.phis[0], spec.kick, 0.05)
    f1, e1 = dm_oracle.device_folded_sweep(L, T, spec.hs[0], spec.phis[0], spec.kick, dev)
    np.testing.assert_allclose(f1, f0, atol=1e-13)
    np.testing.assert_allclose(e1, e0, atol=1e-13)


def test_device_channel_trace_preserving(pkg):
    L = 3
    dev = harsh_device(pkg, L)
    rho = dm_oracle.DM(L, np.eye(1 << L, dtype=np.complex128) / (1 << L))
    rng = np.random.default_rng(1)
    U = np.linalg.qr(rng.normal(size=(8, 8)) + 1j * rng.normal(size=(8, 8)))[0]
    rho = dm_oracle.DM(L, U @ np.diag(rng.random(8) / 4) @ U.conj().T)
    tr0 = np.trace(rho.matrix())
    for i, chn in enumerate(dev.site_channels()):
        dm_oracle.device_channel(rho, i, *chn)
    assert abs(np.trace(rho.matrix()) - tr0) < 1e-14


@pytest.mark.parametrize("state,pol", [("vacuum", "x"), ("neel", "xy")])
def test_importance_weighted_trajectories_match_exact(pkg, state, pol):
    rng = np.random.default_rng(11)
    L, T = 4, 6
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.9, polarization=pol,
                         initial_state=state, device=harsh_device(pkg, L))
    fe, ee = dm_oracle.device_folded_sweep(L, T, spec.hs[0], spec.phis[0], spec.kick,
                                           spec.device, initial_state=state)
    n = 6000
    out = c_oracle.autocorr(spec, n, seed=99)
    for key, exact in (("fwd", fe), ("echo", ee)):
        a = out[key][0]
        mean = a.mean(axis=0)
        se = a.std(axis=0, ddof=1) / np.sqrt(n) + 1e-12
        z = (mean - exact) / se
        assert np.max(np.abs(z)) < 4.5, (key, mean, exact, z)


def test_device_oracle_thread_independent(pkg):
    rng = np.random.default_rng(5)
    L, T = 5, 4
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, device=harsh_device(pkg, L))
    a = c_oracle.autocorr(spec, 16, seed=4, n_threads=1)
    b = c_oracle.autocorr(spec, 16, seed=4, n_threads=4)
    for k in a:
        assert np.array_equal(a[k], b[k])


def test_standin_calibration(pkg):
    cal = pkg.DeviceCalibration.from_json(os.path.join(ROOT, "data", "device_standin_L20.json"))
    assert len(cal.qubits) == 21
    dev = cal.device_noise(20)
    assert dev.L == 20 and dev.gate_ns == 120.0
    q = cal.qubits[1]
    assert dev.p_gate[0] == pytest.approx(2 * (2 * q["sx_error"]))   # 2 sx, p = 2 e
    assert np.all(dev.t2_us <= 2 * dev.t1_us)
    p1 = 2 * cal.qubits[0]["sx_error"]
    p2 = 4 * cal.cz_error / 3
    assert dev.anc_factor == pytest.approx((1 - p1) ** 6 * (1 - p2) ** 2)
    ch = dev.site_channels()
    assert all(0 < g < 1e-3 and 0 <= d < 1e-3 for g, d, _ in ch)
    with pytest.raises(ValueError):
        cal.device_noise(21)


# ---- energy path under device-like noise (energy-fakebrisbane.py) ---------------

def test_readout_observables_exact(pkg):
    """The affine read-out map on Z, ZZ equals flipping every measured bit of an
    arbitrary distribution independently (p01: 0 -> 1, p10: 1 -> 0)."""
    rng = np.random.default_rng(4)
    L = 3
    prob = rng.random(1 << L)
    prob /= prob.sum()
    p01, p10 = np.array([0.02, 0.05, 0.01]), np.array([0.03, 0.01, 0.07])
    flip = np.zeros((1 << L, 1 << L))   # flip[y, x] = P(read y | state x)
    for xs in range(1 << L):
        for ys in range(1 << L):
            pr = 1.0
            for i in range(L):
                bx, by = (xs >> i) & 1, (ys >> i) & 1
                pr *= (p01[i] if by else 1 - p01[i]) if bx == 0 else (1 - p10[i] if by else p10[i])
            flip[ys, xs] = pr
    read = flip @ prob
    zs = lambda d, i: sum(d[x] * (1 - 2 * ((x >> i) & 1)) for x in range(1 << L))
    zzs = lambda d, i: sum(d[x] * (1 - 2 * ((x >> i) & 1)) * (1 - 2 * ((x >> (i + 1)) & 1))
                           for x in range(1 << L))
    obs = {"z": np.array([zs(prob, i) for i in range(L)]),
           "zz": np.array([zzs(prob, i) for i in range(L - 1)]), "x": np.zeros(L)}
    got = pkg.energy.readout_observables(obs, p01, p10)
    np.testing.assert_allclose(got["z"], [zs(read, i) for i in range(L)], atol=1e-15)
    np.testing.assert_allclose(got["zz"], [zzs(read, i) for i in range(L - 1)], atol=1e-15)
    np.testing.assert_allclose(got["x"], p10 - p01, atol=1e-15)


def test_oracle_init_mask_matches_restatement(pkg):
    from oracle import energy_oracle

    rng = np.random.default_rng(2)
    hs, phis = random_disorder(rng, 7)
    spec = pkg.SweepSpec(L=7, T=2, hs=hs, phis=phis, g=0.9, noise_prob=0.4, initial_state="neel")
    import dataclasses

    plain = dataclasses.replace(spec)
    plain.device = None
    for tr in range(40):
        assert c_oracle.init_mask(plain, 17, tr) == energy_oracle.prep_mask(plain, 17, tr)


@pytest.mark.parametrize("state", ["vacuum", "neel"])
def test_energy_oracle_device_trajectories_match_exact(pkg, state):
    """Kraus-weighted energy trajectories of the oracle average to the exact
    density matrix of the device-like channel (Z, ZZ, X every period)."""
    from oracle import energy_oracle

    rng = np.random.default_rng(21)
    L, T, n = 5, 5, 3000
    hs, phis = random_disorder(rng, L)
    spec = pkg.energy.energy_spec(L, T, hs, phis, 0.93, state)
    spec.device = harsh_device(pkg, L)
    exact = dm_oracle.energy_sweep(L, T, hs[0], phis[0], spec.kick, 0.0, initial_state=state,
                                   dev=spec.device)
    runs = [energy_oracle.trajectory_energy(spec, 0, tr, seed=8) for tr in range(n)]
    for k in range(3):
        v = np.array([r[k] for r in runs])
        mean, sd = v.mean(axis=0), v.std(axis=0) / np.sqrt(n) + 1e-12
        assert np.all(np.abs(mean - exact[k]) < 5 * sd), k
