"""Forward prefix cache (dtc_prefix_build / dtc_autocorr_prefixed; the
optimisation controller's shared t-period states) vs the C oracle.

A prefixed run is the trajectory whose periods 1..n_pre were drawn with the
prefix's seed and everything after (later periods, every echo) with the
run's seed: the oracle composes exactly that from orc_apply_periods, per
trajectory, to 1e-10.  Plus the argument checks that keep a continuation on
the prefix it was built from."""
import numpy as np
import pytest

from oracle import c_oracle
from tests.helpers import random_disorder

pytestmark = pytest.mark.gpu
TOL = 1e-10


def harsh_device(pkg, L):
    return pkg.DeviceNoise(p_gate=np.full(L, 0.02), t1_us=np.linspace(1.5, 3.0, L),
                           t2_us=np.linspace(1.0, 4.0, L), gate_ns=120.0, anc_factor=0.9,
                           readout_p01=0.02, readout_p10=0.035)


def specs(pkg, L, T, n_pre, state, pol, dev, seed):
    rng = np.random.default_rng(seed)
    hs, phis = random_disorder(rng, L)
    g = list(np.linspace(0.9, 0.97, T))
    device = harsh_device(pkg, L) if dev else None
    kw = dict(L=L, hs=hs, phis=phis, noise_prob=0.05, polarization=pol, initial_state=state,
              t_offset=1, device=device)
    return pkg.SweepSpec(T=T, g=g, **kw), pkg.SweepSpec(T=n_pre, g=g[:n_pre], **kw)


@pytest.mark.parametrize("L,T,n_pre,state,pol,dev", [
    (6, 5, 3, "neel", "x", False),
    (13, 4, 2, "vacuum", "xy", False),
    (20, 4, 2, "vacuum", "x", False),
    (7, 4, 2, "neel", "x", True),
])
def test_prefixed_run_matches_oracle(pkg, engine, L, T, n_pre, state, pol, dev):
    spec, pre = specs(pkg, L, T, n_pre, state, pol, dev, L + T)
    n = 3
    s_pre, s_run = 11, 22
    engine.prefix_build(pre, n, n_pre, seed=s_pre)
    t_first = n_pre  # period t + 1 > n_pre
    got = engine.autocorr_prefixed(spec, n, seed=s_run, t_first=t_first)
    j = spec.probe_site
    if dev:
        d = spec.device
        fac, ro_a, ro_b = d.anc_factor, 1 - d.readout_p01 - d.readout_p10, d.readout_p10 - d.readout_p01
    else:
        fac, ro_a, ro_b = (1 - 0.05) ** 6, 1.0, 0.0
    for tr in range(n):
        m = c_oracle.init_mask(spec, s_pre, tr)
        zinit = -1.0 if (m >> j) & 1 else 1.0
        F = np.zeros(1 << L, dtype=np.complex128)
        F[m] = 1.0
        F, _ = c_oracle.apply_periods(spec, F, 1, n_pre, traj=tr, stream=0, seed=s_pre)
        for p in range(n_pre + 1, T + 1):
            F, z = c_oracle.apply_periods(spec, F, p, 1, traj=tr, stream=0, seed=s_run)
            t = p - 1
            if t < t_first:
                continue
            _, ze = c_oracle.apply_periods(spec, F, p, p, inverse=True, traj=tr, stream=1 + t,
                                           seed=s_run)
            assert abs(got["fwd"][0, tr, t] - (ro_a * fac * zinit * z[1 + j] + ro_b)) < TOL
            assert abs(got["echo"][0, tr, t] - (ro_a * fac * zinit * ze[1 + j] + ro_b)) < TOL
        assert np.all(got["fwd"][0, tr, :t_first] == 0)
    engine.prefix_release()


def test_prefix_argument_checks(pkg, engine):
    capi = pkg._capi
    spec, pre = specs(pkg, 8, 4, 2, "vacuum", "x", False, 5)
    with pytest.raises(capi.DtcError):
        engine.autocorr_prefixed(spec, 2, seed=1, t_first=2)      # nothing built yet
    engine.prefix_build(pre, 2, 2, seed=3)
    with pytest.raises(capi.DtcError):
        engine.autocorr_prefixed(spec, 3, seed=1, t_first=2)      # other trajectories
    with pytest.raises(capi.DtcError):
        engine.autocorr_prefixed(spec, 2, seed=1, t_first=1)      # measures inside the prefix
    other = pkg.SweepSpec(L=8, T=4, hs=spec.hs, phis=spec.phis, g=[0.8, 0.9, 0.95, 0.97],
                          noise_prob=0.05, t_offset=1)
    with pytest.raises(capi.DtcError):
        engine.autocorr_prefixed(other, 2, seed=1, t_first=2)     # different kick rows
    out = engine.autocorr_prefixed(spec, 2, seed=1, t_first=2)
    assert np.all(np.abs(out["echo"][0, :, 2:]) <= 1.0)
    engine.prefix_release()


def test_optimizer_with_and_without_prefix(pkg, engine):
    """The optimisation loop with the prefix cache (default) and without:
    the same g range and both echoes within shot noise of each other at t=0."""
    ct = pkg.control
    rng = np.random.default_rng(1)
    hs, phis = random_disorder(rng, 10)
    res = {}
    for pc in (1, 0):
        cfg = ct.ControllerConfig(use_optimization=1, prefix_cache=pc, g_max=1.0)
        res[pc] = ct.realtime_adaptive(10, 4, hs, phis, 0.84, cfg, shots=512, engine=engine,
                                       seed=7)
        assert np.all((res[pc].g >= 0.84) & (res[pc].g <= 1.0))
    # t = 0 uses no prefix: same seeds, identical estimate
    assert res[1].echo[0, 0] == res[0].echo[0, 0]
