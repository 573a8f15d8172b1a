"""Pin the oracles before trusting them (CPU only).

1. Exact density-matrix restatement == literal (L+1)-qubit transpiled circuit
   (the folding of SURVEY.md §0.6), noisy and noiseless, fwd and echo, vacuum
   and neel, x and xy kicks.
2. Known answers for hs_L4/phis_L4 row 0.
3. The reference's own committed 1024-shot Aer outputs for L=4
   (autocorr_data_L4/*gain0.0{1,5}.csv, columns av_autocorr_standard /
   av_autocorr_echo_standard: g=0.84, p=0.05, t+1 periods) agree with the
   exact values within shot noise.
4. The C restatement (oracle/dtc_oracle.c): noiseless == exact to 1e-12,
   trajectory means converge to the exact noisy values.
5. The C oracle's Philox4x32-10 reproduces the Random123 known-answer vectors.
"""
import numpy as np
import pytest

from oracle import c_oracle, dm_oracle
from tests.helpers import chi2_per_dof, random_disorder, shot_sigma

# SURVEY.md Appendix B (12 digits), hs_L4/phis_L4 row 0, L=4, j=2
KAT_FWD_P0 = [1.000000000000, -0.995561964603, 0.987503522353, -0.989468190182,
              0.971907601318, -0.987905665657, 0.980562315534, -0.993527511911,
              0.997970723687, -0.996428249419, 0.993891423466, -0.991502810001,
              0.975341292458, -0.987461283389, 0.974943150508, -0.991408279461,
              0.993565855510, -0.996473189390, 0.998333562322, -0.993725951291]
KAT_FWD_P05 = [0.735091890625, -0.695238050455, 0.655287339066, -0.623514561517,
               0.583153523493, -0.561522812377, 0.530792486099, -0.508711963295,
               0.484748742415, -0.459695352029, 0.435622281978, -0.413440907928,
               0.389200901867, -0.372116274863, 0.351275063724, -0.336231492796,
               0.319692346582, -0.304006700393, 0.288962218248, -0.273937562346]
KAT_ECHO_P05 = [0.735091890625, 0.663420431289, 0.598388358974, 0.539522661507,
                0.485984894637, 0.437638990422, 0.394317535877, 0.355379719159,
                0.320525023135, 0.289154722487, 0.260815875590, 0.235211236936,
                0.212032622395, 0.191140367658, 0.172325574032, 0.155387431519,
                0.140196413303, 0.126504829611, 0.114158540595, 0.103007270308]
KAT_CTRL_FWD = [-0.611957637491, 0.459808578785, -0.464011353702, 0.241187894719,
                -0.395014825237, 0.367167602612, -0.387899608426, 0.378426821327,
                -0.347634034083, 0.258314059073, -0.295837534474, 0.246477172983,
                -0.256745970846, 0.235363698725, -0.227167453405, 0.179817795155,
                -0.205600147348, 0.173366865350, -0.185941610477, 0.177413055068]
KAT_CTRL_ECHO = [0.663420431289, 0.589576316167, 0.519480336946, 0.448920600020,
                 0.383964251348, 0.334063523155, 0.290473719439, 0.253653234249,
                 0.222581842050, 0.194431672765, 0.169313202368, 0.148735156674,
                 0.130056165849, 0.114458922154, 0.100872690713, 0.088706054320,
                 0.078443203083, 0.069895048045, 0.062069569070, 0.055576693603]


@pytest.fixture(scope="module")
def l4(golden):
    d = golden["disorder"]["L4"]
    return np.array(d["hs"])[0, :4], np.array(d["phis"])[0, :3]


@pytest.mark.parametrize("p,state,pol", [(0.0, "vacuum", "x"), (0.05, "vacuum", "x"),
                                         (0.05, "neel", "x"), (0.1, "vacuum", "xy"),
                                         (0.05, "neel", "circular_left")])
def test_folding_equals_ancilla_circuit(pkg, l4, p, state, pol):
    hs, phis = l4
    L, T = 4, 5
    kick = pkg.kick_table(L, T, 0.97, pol)
    fwd, echo = dm_oracle.folded_sweep(L, T, hs, phis, kick, p, initial_state=state)
    for t in range(T):
        a = dm_oracle.ancilla_circuit_expectation(L, t, hs, phis, kick, p, echo=False,
                                                  initial_state=state)
        b = dm_oracle.ancilla_circuit_expectation(L, t, hs, phis, kick, p, echo=True,
                                                  initial_state=state)
        assert abs(a - fwd[t]) < 1e-12
        assert abs(b - echo[t]) < 1e-12


def test_folding_L6_neel_odd_probe(pkg, golden):
    # L=6: j=3 is flipped by the neel prep (its noisy X enters the sign)
    d = golden["disorder"]["L6"]
    hs, phis = np.array(d["hs"])[0], np.array(d["phis"])[0]
    kick = pkg.kick_table(6, 3, 0.9, "x")
    fwd, echo = dm_oracle.folded_sweep(6, 3, hs, phis, kick, 0.05, initial_state="neel")
    for t in range(3):
        a = dm_oracle.ancilla_circuit_expectation(6, t, hs, phis, kick, 0.05,
                                                  initial_state="neel")
        b = dm_oracle.ancilla_circuit_expectation(6, t, hs, phis, kick, 0.05, echo=True,
                                                  initial_state="neel")
        assert abs(a - fwd[t]) < 1e-12 and abs(b - echo[t]) < 1e-12


def test_known_answers_appendix_b(pkg, l4):
    hs, phis = l4
    f0, e0 = dm_oracle.folded_sweep(4, 20, hs, phis, pkg.kick_table(4, 19, 0.97), 0.0)
    np.testing.assert_allclose(f0, KAT_FWD_P0, atol=1e-11)
    np.testing.assert_allclose(e0, np.ones(20), atol=1e-12)
    f, e = dm_oracle.folded_sweep(4, 20, hs, phis, pkg.kick_table(4, 19, 0.97), 0.05)
    np.testing.assert_allclose(f, KAT_FWD_P05, atol=1e-11)
    np.testing.assert_allclose(e, KAT_ECHO_P05, atol=1e-11)
    fc, ec = dm_oracle.folded_sweep(4, 20, hs, phis, pkg.kick_table(4, 20, 0.84), 0.05,
                                    t_offset=1)
    np.testing.assert_allclose(fc, KAT_CTRL_FWD, atol=1e-11)
    np.testing.assert_allclose(ec, KAT_CTRL_ECHO, atol=1e-11)


def test_analytic_t0_t1(pkg, l4):
    hs, phis = l4
    p, g = 0.05, 0.97
    f, e = dm_oracle.folded_sweep(4, 2, hs, phis, pkg.kick_table(4, 1, g), p)
    assert abs(f[0] - (1 - p) ** 6) < 1e-14 and abs(e[0] - (1 - p) ** 6) < 1e-14
    assert abs(f[1] - (1 - p) ** 7 * np.cos(np.pi * g)) < 1e-12
    assert abs(e[1] - (1 - p) ** 8) < 1e-12


@pytest.mark.parametrize("gain", ["0.01", "0.05"])
def test_exact_vs_reference_aer_csv_L4(pkg, l4, golden, gain):
    """The reference's committed Aer outputs (1024 shots) vs the exact values."""
    case = [c for c in golden["aer_autocorr"] if c["name"] == f"L4_ctrl_standard_gain{gain}"][0]
    hs, phis = l4
    T = len(case["time"])
    fc, ec = dm_oracle.folded_sweep(4, T, hs, phis, pkg.kick_table(4, T, 0.84), 0.05,
                                    t_offset=1)
    for key, exact in (("fwd", fc), ("echo", ec)):
        ref = np.array(case["columns"][key])
        assert np.all(np.abs(ref * 512 - np.round(ref * 512)) < 1e-9)  # 1024-shot values
        chi2, zmax = chi2_per_dof(ref, exact, shot_sigma(exact), 0.0)
        assert chi2 < 2.0 and zmax < 4.0, (key, chi2, zmax)


@pytest.mark.parametrize("state,pol", [("vacuum", "x"), ("neel", "x"), ("vacuum", "xy")])
def test_c_oracle_noiseless_exact(pkg, l4, state, pol):
    hs, phis = l4
    spec = pkg.SweepSpec(L=4, T=12, hs=hs[None], phis=phis[None], g=0.97, polarization=pol,
                         initial_state=state, noise_prob=0.0, use_noise=0)
    out = c_oracle.autocorr(spec, 1)
    f, e = dm_oracle.folded_sweep(4, 12, hs, phis, spec.kick, 0.0, initial_state=state)
    np.testing.assert_allclose(out["fwd"][0, 0], f, atol=1e-12)
    np.testing.assert_allclose(out["echo"][0, 0], e, atol=1e-12)


@pytest.mark.parametrize("state,pol,toff", [("vacuum", "x", 0), ("neel", "x", 0),
                                            ("vacuum", "circular_right", 0),
                                            ("vacuum", "x", 1)])
def test_c_oracle_trajectories_converge(pkg, l4, state, pol, toff):
    hs, phis = l4
    T, n = 10, 6000
    spec = pkg.SweepSpec(L=4, T=T, hs=hs[None], phis=phis[None], g=0.97, polarization=pol,
                         initial_state=state, noise_prob=0.08, t_offset=toff)
    out = c_oracle.autocorr(spec, n, seed=11)
    f, e = dm_oracle.folded_sweep(4, T, hs, phis, spec.kick, 0.08, initial_state=state,
                                  t_offset=toff)
    for key, exact in (("fwd", f), ("echo", e)):
        a = out[key][0]
        se = a.std(axis=0) / np.sqrt(n) + 1e-12
        z = np.abs(a.mean(axis=0) - exact) / se
        z = z[a.std(axis=0) > 1e-9]
        assert np.max(z) < 4.5, (key, z)


def _philox_py(ctr, key):
    M0, M1, W0, W1 = 0xD2511F53, 0xCD9E8D57, 0x9E3779B9, 0xBB67AE85
    c = list(ctr)
    k0, k1 = key
    for _ in range(10):
        p0, p1 = M0 * c[0], M1 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k0) & 0xFFFFFFFF, p1 & 0xFFFFFFFF,
             ((p0 >> 32) ^ c[3] ^ k1) & 0xFFFFFFFF, p0 & 0xFFFFFFFF]
        k0, k1 = (k0 + W0) & 0xFFFFFFFF, (k1 + W1) & 0xFFFFFFFF
    return c


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert _philox_py([0, 0, 0, 0], [0, 0]) == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]
    assert _philox_py([0xFFFFFFFF] * 4, [0xFFFFFFFF] * 2) == \
        [0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD]
    assert _philox_py([0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344],
                      [0xA4093822, 0x299F31D0]) == [0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1]


def test_oracle_pauli_sampling_contract():
    """orc_sample_pauli == thresholds on Philox word 0 (include/dtc.h contract)."""
    p, seed = 0.05, 0x5EED0001
    thr = [int(np.floor(k * p / 4 * 2**32 + 0.5)) for k in (1, 2, 3)]
    rng = np.random.default_rng(3)
    for _ in range(300):
        traj = int(rng.integers(0, 2**40))
        stream, period, site, sub = (int(x) for x in rng.integers(0, 50, 4))
        w = _philox_py([site | (sub << 16), period, stream, traj & 0xFFFFFFFF],
                       [seed & 0xFFFFFFFF, ((seed >> 32) ^ (traj >> 32)) & 0xFFFFFFFF])[0]
        want = 1 if w < thr[0] else 2 if w < thr[1] else 3 if w < thr[2] else 0
        assert c_oracle.sample_pauli(p, seed, traj, stream, period, site, sub) == want
    # empirical rates over many draws
    draws = np.array([c_oracle.sample_pauli(0.2, 1, t, 0, 1, 2, 0) for t in range(20000)])
    for code in (1, 2, 3):
        assert abs(np.mean(draws == code) - 0.05) < 0.006


def test_c_oracle_apply_periods_inverse_roundtrip(pkg):
    rng = np.random.default_rng(5)
    L = 7
    hs, phis = random_disorder(rng, L)
    spec = pkg.SweepSpec(L=L, T=6, hs=hs, phis=phis, g=0.93, noise_prob=0.0, use_noise=0,
                         polarization="xy")
    psi = rng.normal(size=1 << L) + 1j * rng.normal(size=1 << L)
    psi /= np.linalg.norm(psi)
    a, _ = c_oracle.apply_periods(spec, psi, 1, 5)
    b, z = c_oracle.apply_periods(spec, a, 5, 5, inverse=True)
    np.testing.assert_allclose(b, psi, atol=1e-12)
    assert abs(z[0] - 1) < 1e-12


def test_blocks_factorise_oracle(pkg):
    """The property tests/test_gpu_large.py relies on at L=28, checked with the
    oracle at L=10: zero couplings on two bonds split the chain, and per-site
    <Z_i(t)> of the full chain equal those of the block holding i."""
    rng = np.random.default_rng(10)
    L, T, g, cuts = 10, 8, 0.93, (3, 6)
    hs = rng.uniform(-np.pi, np.pi, (1, L))
    phis = rng.uniform(-1.5 * np.pi, -0.5 * np.pi, (1, L - 1))
    phis[:, list(cuts)] = 0.0
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=g, polarization="circular_left",
                         initial_state="neel", use_noise=0)
    full = c_oracle.autocorr(spec, 1, want_echo=False, want_zsite=True)["zsite"]
    mask, lo = spec.init_mask, 0
    for hi in (cuts[0] + 1, cuts[1] + 1, L):
        Lb = hi - lo
        b = pkg.SweepSpec(L=Lb, T=T, hs=hs[:, lo:hi], phis=phis[:, lo:hi - 1], g=g,
                          use_noise=0, kick=spec.kick[:, lo:hi],
                          init_mask_value=(mask >> lo) & ((1 << Lb) - 1))
        ref = c_oracle.autocorr(b, 1, want_echo=False, want_zsite=True)["zsite"]
        assert np.abs(full[..., lo:hi] - ref).max() < 1e-12
        lo = hi


@pytest.mark.parametrize("L,T,pol,state,toff,p", [
    (4, 6, "x", "vacuum", 0, 0.07),
    (9, 5, "xy", "neel", 1, 0.07),
    (12, 5, "x", "vacuum", 0, 0.0),
    (13, 5, "circular_left", "neel", 0, 0.05),
    (15, 4, "y", "vacuum", 0, 0.1),
])
def test_fused_cpu_restatement_matches_gate_oracle(pkg, L, T, pol, state, toff, p):
    """bench.py's CPU baseline (orc_autocorr_fused: composed per-site kicks,
    blocked low/high sweeps, table diagonal) runs the same trajectories as the
    gate-by-gate oracle: equal per trajectory to rounding."""
    rng = np.random.default_rng(L)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)
    a = c_oracle.autocorr(spec, 3, seed=5)
    b = c_oracle.autocorr_fused(spec, 3, seed=5)
    assert np.abs(a["fwd"] - b["fwd"]).max() < 1e-12
    assert np.abs(a["echo"] - b["echo"]).max() < 1e-12


def test_large_state_sweep_thread_independent(pkg):
    """States of 2^22 amplitudes and more are swept by all threads, one
    trajectory at a time (the L=28 parity runs, test_gpu_l28_oracle.py): the
    gates are element-wise, so one thread and four give the same trajectory;
    only measure_z's partial sums over 4M amplitudes are grouped differently (1e-11)."""
    L = 22
    rng = np.random.default_rng(5)
    hs, phis = random_disorder(rng, L, 1)
    spec = pkg.SweepSpec(L=L, T=3, hs=hs, phis=phis, g=0.93, noise_prob=0.05,
                         polarization="circular_left", initial_state="neel")
    one = c_oracle.autocorr(spec, 2, seed=9, want_zsite=True, n_threads=1)
    four = c_oracle.autocorr(spec, 2, seed=9, want_zsite=True, n_threads=4)
    for k in one:
        assert np.abs(one[k] - four[k]).max() < 1e-11, k
    # and the same trajectory as the small-state (per-trajectory threaded)
    # path's arithmetic: the fused restatement agrees to 1e-10
    fused = c_oracle.autocorr_fused(spec, 2, seed=9, n_threads=4)
    for k in ("fwd", "echo"):
        assert np.abs(one[k] - fused[k]).max() < 1e-10, k
