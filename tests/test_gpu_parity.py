"""HIP engine (through the C ABI) vs the CPU oracle, per trajectory.

The engine and oracle share the RNG contract of include/dtc.h, so each noisy
trajectory is the same random circuit on both sides: per-trajectory
autocorrelator values must agree to 1e-10 (summation order is the only
difference; observed ~1e-13 at L=20).
"""
import numpy as np
import pytest

from oracle import c_oracle, dm_oracle
from tests.helpers import random_disorder

pytestmark = pytest.mark.gpu
TOL = 1e-10


def _cmp(a, b, tol=TOL):
    for k in b:
        err = float(np.abs(a[k] - b[k]).max())
        assert err < tol, (k, err)


CASES = [
    # L, T, n_inst, n_traj, p, state, pol, t_offset
    # edge sizes: one- to three-site chains (sites 1..11 of the 12-bit tile are
    # padding) and the shortest sweeps (T=1: only t=0; T=2: one period)
    (1, 4, 1, 3, 0.05, "vacuum", "x", 0),
    (2, 5, 2, 3, 0.1, "neel", "xy", 0),
    (3, 6, 1, 4, 0.05, "neel", "circular_left", 1),
    (6, 1, 1, 2, 0.05, "vacuum", "x", 0),
    (6, 2, 1, 3, 0.05, "neel", "x", 1),
    (4, 20, 1, 1, 0.0, "vacuum", "x", 0),
    (4, 12, 1, 6, 0.05, "neel", "x", 0),
    (5, 9, 2, 3, 0.1, "vacuum", "circular_left", 0),
    (8, 9, 1, 4, 0.05, "neel", "yx", 1),
    (11, 8, 1, 3, 0.05, "vacuum", "xy_cycle", 0),
    (12, 8, 2, 3, 0.05, "vacuum", "x", 0),
    (13, 7, 1, 3, 0.2, "neel", "y", 0),
    (15, 6, 1, 2, 0.05, "vacuum", "xy", 1),
    (16, 6, 1, 2, 0.05, "neel", "circular_right", 0),
    (17, 5, 1, 2, 0.05, "vacuum", "x", 0),
    (20, 6, 1, 2, 0.05, "vacuum", "x", 0),
]


@pytest.mark.parametrize("L,T,n_inst,n_traj,p,state,pol,toff", CASES)
def test_engine_matches_oracle(pkg, engine, L, T, n_inst, n_traj, p, state, pol, toff):
    rng = np.random.default_rng(L * 100 + T)
    hs, phis = random_disorder(rng, L, n_inst)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)
    got = engine.autocorr(spec, n_traj, seed=1234, want_zsite=True)
    ref = c_oracle.autocorr(spec, n_traj, seed=1234, want_zsite=True)
    _cmp(got, ref)


def test_per_period_g_list(pkg, engine):
    """controlled-g.py: g_values[step] per period, t+1 periods."""
    rng = np.random.default_rng(3)
    L, T = 10, 8
    hs, phis = random_disorder(rng, L)
    gl = list(np.linspace(0.84, 1.0, T))
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=gl, noise_prob=0.05, t_offset=1)
    _cmp(engine.autocorr(spec, 3, seed=5), c_oracle.autocorr(spec, 3, seed=5))


@pytest.mark.parametrize("L", [4, 9, 12, 14, 18, 20])
@pytest.mark.parametrize("inverse", [False, True])
def test_apply_periods_random_state(pkg, engine, L, inverse):
    rng = np.random.default_rng(L + 7 * inverse)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=5, hs=hs, phis=phis, g=0.97, noise_prob=0.1, polarization="xy")
    psi = rng.normal(size=1 << L) + 1j * rng.normal(size=1 << L)
    psi /= np.linalg.norm(psi)
    first = 3 if inverse else 2
    ga, gz = engine.apply_periods(spec, psi, first, 3, inverse=inverse, inst=1, traj=11,
                                  stream=4, seed=99)
    oa, oz = c_oracle.apply_periods(spec, psi, first, 3, inverse=inverse, inst=1, traj=11,
                                    stream=4, seed=99)
    assert np.abs(ga - oa).max() < 1e-12
    assert np.abs(gz - oz).max() < 1e-11


def test_forward_inverse_roundtrip_noiseless(pkg, engine):
    rng = np.random.default_rng(1)
    L = 20
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=8, hs=hs, phis=phis, g=0.97, noise_prob=0.0, use_noise=0)
    psi = rng.normal(size=1 << L) + 1j * rng.normal(size=1 << L)
    psi /= np.linalg.norm(psi)
    a, za = engine.apply_periods(spec, psi, 1, 7)
    assert abs(za[0] - 1.0) < 1e-12
    b, _ = engine.apply_periods(spec, a, 7, 7, inverse=True)
    assert np.abs(b - psi).max() < 1e-12


def test_noiseless_L20_statevector_oracle(pkg, engine, golden):
    """hs_L20 row 0, g=0.97: forward <Z_i>(t) vs the numpy statevector oracle."""
    d = golden["disorder"]["L20"]
    hs, phis = np.array(d["hs"][:1]), np.array(d["phis"][:1])
    spec = pkg.SweepSpec(L=20, T=10, hs=hs, phis=phis, g=0.97, noise_prob=0.0, use_noise=0)
    out = engine.autocorr(spec, 1, want_zsite=True, want_echo=True)
    z = dm_oracle.statevector_zsite(20, 10, hs[0], phis[0], spec.kick)
    assert np.abs(out["zsite"][0, 0] - z).max() < 1e-10
    np.testing.assert_allclose(out["fwd"][0, 0], z[:, 10], atol=1e-10)
    # <Z_10(t)> for t = 0..3
    np.testing.assert_allclose(z[:4, 10], [1, -0.995562, 0.999894, -0.994949], atol=1e-6)
    np.testing.assert_allclose(out["echo"][0, 0], np.ones(10), atol=1e-10)


@pytest.mark.parametrize("L", [14, 16])
def test_batching_and_sharding_invariance(pkg, engine, L):
    """Per-trajectory values depend only on the global trajectory id.  The full
    batch (12 states) runs in the octet layout, batches of 1 and 5 in the
    contiguous one; at L=16 (16 tiles per state) the contiguous launches also
    take the XCD-aware tile order (each XCD an eighth of a state's tiles)."""
    rng = np.random.default_rng(4)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=6, hs=hs, phis=phis, g=0.9, noise_prob=0.1)
    full = engine.autocorr(spec, 6, seed=21, batch=0)
    b1 = engine.autocorr(spec, 6, seed=21, batch=1)
    b5 = engine.autocorr(spec, 6, seed=21, batch=5)
    lo = engine.autocorr(spec, 2, seed=21, traj_offset=0)
    hi = engine.autocorr(spec, 4, seed=21, traj_offset=2)
    for k in ("fwd", "echo"):
        assert np.array_equal(full[k], b1[k]) and np.array_equal(full[k], b5[k])
        assert np.array_equal(full[k], np.concatenate([lo[k], hi[k]], axis=1))


def test_t_first_single_time_point(pkg, engine):
    rng = np.random.default_rng(6)
    hs, phis = random_disorder(rng, 12)
    spec = pkg.SweepSpec(L=12, T=7, hs=hs, phis=phis, noise_prob=0.05)
    full = engine.autocorr(spec, 3, seed=8)
    last = engine.autocorr(spec, 3, seed=8, t_first=6)
    for k in ("fwd", "echo"):
        assert np.array_equal(full[k][..., 6], last[k][..., 6])
        assert not np.any(last[k][..., :6])


def test_error_paths(pkg, engine):
    rng = np.random.default_rng(0)
    hs, phis = random_disorder(rng, 6)
    spec = pkg.SweepSpec(L=6, T=4, hs=hs, phis=phis)
    with pytest.raises(pkg._capi.DtcError, match="n_traj"):
        engine.autocorr(spec, 0)
    bad = pkg.SweepSpec(L=6, T=4, hs=hs, phis=phis, probe_site=6)
    with pytest.raises(pkg._capi.DtcError, match="probe_site"):
        engine.autocorr(bad, 1)
    with pytest.raises(pkg._capi.DtcError, match="period range"):
        engine.apply_periods(spec, np.eye(1, 64)[0], 3, 4)


def test_distribution_statistics_L8(pkg, engine):
    """Trajectory means vs the exact noisy density matrix (z-test)."""
    rng = np.random.default_rng(12)
    L, T, n = 8, 8, 4096
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.95, noise_prob=0.05,
                         initial_state="neel")
    out = engine.autocorr(spec, n, seed=2024)
    f, e = dm_oracle.folded_sweep(L, T, hs[0], phis[0], spec.kick, 0.05, initial_state="neel")
    for key, exact in (("fwd", f), ("echo", e)):
        a = out[key][0]
        sd = a.std(axis=0)
        ok = sd > 1e-9
        z = np.abs(a.mean(axis=0) - exact)[ok] / (sd[ok] / np.sqrt(n))
        assert np.allclose(a.mean(axis=0)[~ok], exact[~ok], atol=1e-12)
        assert z.max() < 4.5, (key, z)


def test_noise_sampler_unbiased_high_resolution(pkg, engine):
    """2^22 trajectories at L=12, T=2 (sub-0.5 % resolution on the sampler).

    t = 1 forward: RX(pi g) then one Pauli draw on the probe site; X or Y flips
    <Z_j>, so every trajectory's value is +-(1-p)^6 cos(pi g), flipped with
    probability exactly p/2 (I, Z keep it) -- a binomial count.  Echo t = 1:
    the mean is (1-p)^8.  A 1 % bias in the Pauli sampler would
    be ~4 sigma on the flip count and ~15 sigma on the echo."""
    from scipy import stats

    L, p, g, n = 12, 0.05, 0.97, 1 << 22
    rng = np.random.default_rng(12)
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=2, hs=hs, phis=phis, g=g, noise_prob=p)
    out = engine.autocorr(spec, n, seed=0xB1A5, batch=32768)
    fwd1, echo1 = out["fwd"][0, :, 1], out["echo"][0, :, 1]
    base = (1 - p) ** 6 * np.cos(np.pi * g)
    assert np.abs(np.abs(fwd1) - abs(base)).max() < 1e-12      # every value is +-base
    flips = int(np.count_nonzero(np.sign(fwd1) != np.sign(base)))
    pval = stats.binomtest(flips, n, p / 2).pvalue
    assert pval > 1e-4, (flips / n, p / 2, pval)
    assert abs(flips / n / (p / 2) - 1) < 0.01                # within 1 % of p/2
    m, se = echo1.mean(), echo1.std() / np.sqrt(n)
    assert abs(m - (1 - p) ** 8) < 4.5 * se, (m, (1 - p) ** 8, se)
    assert se / (1 - p) ** 8 < 5e-4


@pytest.mark.parametrize("L,T,p,state,pol,toff,probe,wide", [
    # wide: the 10-site window merges five passes somewhere (True), or the
    # layers do not fit it and every chain keeps the 8-site form (False)
    (20, 7, 0.1, "vacuum", "x", 0, None, True),
    (20, 6, 0.05, "neel", "xy", 1, None, False),        # general kicks: no light cone
    (21, 6, 0.1, "vacuum", "circular_left", 0, None, False),
    (21, 5, 0.0, "vacuum", "y", 0, None, None),
    (12, 6, 0.1, "vacuum", "x", 0, None, None),
    (14, 7, 0.1, "neel", "y", 0, None, True),
    (16, 6, 0.1, "vacuum", "x", 0, 5, False),            # j - 4 < 2
    (18, 6, 0.1, "vacuum", "x", 1, 13, True),
    (22, 8, 0.05, "vacuum", "y", 0, None, False),        # three site groups
    # edges: j - 4 = 2 with the first layer's group spanning sites 1 .. 11 (11
    # sites: too wide), j + 3 = L - 1, and a 9-site second group (L = 21:
    # 128-B columns), with t_offset and RY kicks
    (16, 7, 0.1, "neel", "x", 0, 6, False),
    (16, 7, 0.1, "vacuum", "y", 1, 12, True),
    (21, 7, 0.1, "vacuum", "y", 0, None, True),
])
def test_echo_light_cone_end(pkg, monkeypatch, L, T, p, state, pol, toff, probe, wide):
    """Echo chains ending in the light-cone pass (the chain's last passes merged
    into one measure-only pass, each kick layer cut to the light cone of Z_j):
    five passes over a 10-site window (dtc_lcw2_final) where it fits, else four
    over an 8-site window (DTC_NO_LCW=1 forces the latter everywhere).  Both
    give the same per-trajectory echo as the oracle (1e-10) and as the engine
    without the merge (DTC_NO_LIGHTCONE=1); pass counts are taken with the
    dual pass off (DTC_NO_DUAL=1) and the 10-site window's (DTC_NO_LCW3=1:
    test_lcw3_c2_form covers the 12-site one).  The options are read when an
    engine opens, so each variant runs on its own engine."""
    rng = np.random.default_rng(L * 31 + T)
    hs, phis = random_disorder(rng, L, 2)
    kw = {} if probe is None else {"probe_site": probe}
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff, **kw)

    def run(env):
        with monkeypatch.context() as m:
            for k in env:
                m.setenv(k, "1")
            with pkg.DtcEngine(0) as eng:
                eng.set_profiling(True)
                out = eng.autocorr(spec, 3, seed=77)
                st = eng.kernel_stats()
        return out, st[pkg._capi.KERNEL_LO_PASS]["launches"] + st[pkg._capi.KERNEL_HI_PASS]["launches"]

    got, _ = run([])
    ref = c_oracle.autocorr(spec, 3, seed=77)
    _cmp(got, ref)
    # pass counts without the dual forward+echo-start pass, which also removes
    # passes (the chain's first) and so blurs the light-cone saving
    single, n_wide = run(["DTC_NO_DUAL", "DTC_NO_LCW3"])
    narrow, n_narrow = run(["DTC_NO_LCW", "DTC_NO_DUAL"])
    full, n_full = run(["DTC_NO_LIGHTCONE", "DTC_NO_DUAL"])
    for o in (single, narrow, full):
        assert np.abs(got["echo"] - o["echo"]).max() < 1e-12
        # (these run without the dual pass, whose forward tile shares its
        # kernel with the echo's: the compiler may contract its FMAs
        # differently, 1e-17 here, as in test_dual_pass_echo_start)
        assert np.abs(got["fwd"] - o["fwd"]).max() < 1e-13
    assert n_wide <= n_narrow <= n_full
    if pol in ("x", "y"):  # factored kicks (general 2x2 kicks keep the full passes)
        assert n_narrow < n_full
    if wide is not None:
        assert (n_wide < n_narrow) == wide, (n_wide, n_narrow)


@pytest.mark.parametrize("L,pol,state,toff,g,p", [
    (20, "x", "vacuum", 0, 0.97, 0.05),   # BASELINE configs[1]'s kicks and noise
    (20, "y", "neel", 1, 0.93, 0.1),
    (21, "x", "neel", 0, 0.91, 0.1),      # 12 + 9 sites: 128-B columns in the forward passes
    (21, "y", "vacuum", 1, 0.97, 0.0),    # noiseless: identity frames
])
def test_lcw2_c2_form(pkg, monkeypatch, L, pol, state, toff, g, p):
    """The C2 chains' 10-site light-cone end runs as dtc_lcw2_final (three LDS
    re-layouts, row swaps, pre-masked cone tables): its launches are counted
    (dtc_lightcone_counts) and its echo equals the C oracle per trajectory
    (1e-10) and the 8-site form (DTC_NO_LCW) to 1e-12."""
    rng = np.random.default_rng(L * 7 + toff)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=9, hs=hs, phis=phis, g=g, noise_prob=p, use_noise=int(p > 0),
                         polarization=pol, initial_state=state, t_offset=toff)
    with monkeypatch.context() as m:
        m.setenv("DTC_NO_LCW3", "1")  # the 10-site ends only
        with pkg.DtcEngine(0) as eng:
            got = eng.autocorr(spec, 3, seed=91)
            counts = eng.lightcone_counts()
    assert counts["lcw2"] > 0 and counts["lcw"] == 0 and counts["lcw3"] == 0, counts
    _cmp(got, c_oracle.autocorr(spec, 3, seed=91))
    with monkeypatch.context() as m:
        m.setenv("DTC_NO_LCW", "1")
        with pkg.DtcEngine(0) as eng:
            narrow = eng.autocorr(spec, 3, seed=91)
            assert eng.lightcone_counts()["lcw2"] == 0
    assert np.abs(got["echo"] - narrow["echo"]).max() < 1e-12


@pytest.mark.parametrize("L,T,pol,state,toff,p", [
    (20, 12, "x", "vacuum", 0, 0.05),     # C2's kicks: 12 + 8 site groups
    (16, 10, "y", "neel", 1, 0.1),
    (13, 9, "circular_left", "vacuum", 0, 0.1),   # general 2x2 kicks
    (22, 8, "x", "neel", 0, 0.05),        # three site groups
])
def test_dual_pass_echo_start(pkg, monkeypatch, L, T, pol, state, toff, p):
    """An echo chain's first pass folded into the forward K-D-K before it
    (dtc_kdk_dual: the tile after the pre-kick K_p also takes the chain's first
    inverse layer and goes to E, since undo(K_{p+1}) D^* D K_p = K_p): per
    trajectory the oracle's values (1e-10), the unfused schedule's
    (DTC_NO_DUAL) to 1e-12, and fewer K-D-K launches."""
    rng = np.random.default_rng(L * 5 + T)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)

    def run(no_dual):
        with monkeypatch.context() as m:
            if no_dual:
                m.setenv("DTC_NO_DUAL", "1")
            with pkg.DtcEngine(0) as eng:
                eng.set_profiling(True)
                out = eng.autocorr(spec, 3, seed=19)
                st = eng.kernel_stats()
        return out, st[pkg._capi.KERNEL_LO_PASS]

    got, lo = run(False)
    ref, lo_ref = run(True)
    _cmp(got, c_oracle.autocorr(spec, 3, seed=19))
    assert np.abs(got["echo"] - ref["echo"]).max() < 1e-12
    assert np.abs(got["fwd"] - ref["fwd"]).max() < 1e-13
    assert lo["launches"] < lo_ref["launches"], (lo, lo_ref)
    # a dual pass moves 48 B per amplitude, 16 fewer than its two passes
    # (2 instances x 3 trajectories per launch)
    n_dual = lo_ref["launches"] - lo["launches"]
    assert lo["bytes"] == pytest.approx(lo_ref["bytes"] - n_dual * 16.0 * 6 * (1 << max(L, 12)))


def test_independent_t_matches_oracle(pkg, engine):
    """--independent_t: every t from its own trajectories (t_first runs of
    t + t_offset periods, fast.py:219-221) -- engine = C oracle per trajectory."""
    from oracle import c_oracle

    rng = np.random.default_rng(31)
    L, T, n = 13, 6, 4
    hs = rng.uniform(-np.pi, np.pi, (1, L))
    phis = rng.uniform(-1.5 * np.pi, -0.5 * np.pi, (1, L - 1))
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=0.07,
                         initial_state="neel", polarization="xy")

    class Oracle:
        def autocorr(self, spec, n_traj, seed=0x5EED0001, traj_offset=0, want_fwd=True,
                     want_echo=True, want_zsite=False, batch=0, t_first=0):
            return c_oracle.autocorr(spec, n_traj, seed=seed, traj_offset=traj_offset,
                                     want_fwd=want_fwd, want_echo=want_echo, t_first=t_first)

    got = pkg.sweep.autocorr_independent_t(engine, spec, n, seed=5)
    ref = pkg.sweep.autocorr_independent_t(Oracle(), spec, n, seed=5)
    for k in ("fwd", "echo"):
        assert np.abs(got[k] - ref[k]).max() < 1e-10



@pytest.mark.parametrize("L,T,pol,state,toff,g,p", [
    (20, 12, "x", "vacuum", 0, 0.97, 0.05),   # BASELINE configs[1]'s kicks and noise
    (20, 10, "y", "neel", 1, 0.93, 0.1),
    (21, 11, "x", "neel", 0, 0.91, 0.1),      # 12 + 9 sites
    (22, 10, "x", "vacuum", 0, 0.95, 0.05),   # three site groups: the form may not fit
    (20, 9, "y", "vacuum", 1, 0.97, 0.0),     # noiseless: identity frames
])
def test_lcw3_c2_form(pkg, monkeypatch, L, T, pol, state, toff, g, p):
    """The 12-site light-cone end (dtc_lcw3_final: the chain's last six passes
    as seven layers over j-5 .. j+6, no column bits): where it runs, the echo
    equals the C oracle per trajectory (1e-10), the 10-site ends
    (DTC_NO_LCW3) and the 8-site ones (DTC_NO_LCW) to 1e-12, with fewer pass
    launches than the 10-site form; the forward values are unchanged."""
    rng = np.random.default_rng(L * 11 + T)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=g, noise_prob=p, use_noise=int(p > 0),
                         polarization=pol, initial_state=state, t_offset=toff)

    def run(env):
        with monkeypatch.context() as m:
            for k in env:
                m.setenv(k, "1")
            with pkg.DtcEngine(0) as eng:
                eng.set_profiling(True)
                out = eng.autocorr(spec, 3, seed=57)
                st = eng.kernel_stats()
                counts = eng.lightcone_counts()
        n = st[pkg._capi.KERNEL_LO_PASS]["launches"] + st[pkg._capi.KERNEL_HI_PASS]["launches"]
        return out, counts, n

    got, counts, n3 = run([])
    _cmp(got, c_oracle.autocorr(spec, 3, seed=57))
    w10, c10, n10 = run(["DTC_NO_LCW3"])
    w8, _, _ = run(["DTC_NO_LCW"])
    for o in (w10, w8):
        assert np.abs(got["echo"] - o["echo"]).max() < 1e-12
        # the forward pass that carries a chain's echo start is a dual pass in
        # one schedule and a plain K-D-K in the other; the 8-site dual runs its
        # kicks in Pauli-frame form and the plain 8-site pass in branch form
        # (round 6), so the forward may differ by an ulp (as in
        # test_echo_light_cone_end)
        assert np.abs(got["fwd"] - o["fwd"]).max() < 1e-13
    assert c10["lcw3"] == 0
    if L <= 21:  # two site groups: the C2 chains' form
        assert counts["lcw3"] > 0, counts
        assert n3 < n10, (n3, n10)
    else:
        assert n3 <= n10
