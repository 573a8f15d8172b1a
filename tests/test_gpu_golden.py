"""HIP engine vs the reference's committed Aer outputs (1024-shot CSVs).

Each golden value is a 1024-shot estimate (sigma = sqrt(1-A^2)/32); the
engine's value is a trajectory mean with its own standard error.  Criterion
per series: chi^2/dof < 2 and every |z| < 4.5.  These pin
the noise model, the transpiled noise placement, the kick variants (x, y,
xy, yx, circular_left/right), the t+1 convention of the controlled-g
scripts and the disorder rows.
"""
import numpy as np
import pytest

from oracle import dm_oracle
from tests.helpers import chi2_per_dof, shot_sigma

pytestmark = pytest.mark.gpu

N_TRAJ = 2048


def _cases(golden, prefix):
    return [c for c in golden["aer_autocorr"] if c["name"].startswith(prefix)]


def _run_case(pkg, engine, golden, case, n_traj=N_TRAJ):
    cfg = case["config"]
    L = cfg["L"]
    d = golden["disorder"][f"L{L}"]
    r = cfg["inst_row"]
    hs, phis = np.array(d["hs"][r:r + 1]), np.array(d["phis"][r:r + 1])
    T = len(case["time"])
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=cfg["g"],
                         polarization=cfg["polarization"],
                         circular_frequency=cfg.get("circular_frequency", 1.0),
                         initial_state=cfg["initial_state"], noise_prob=cfg["noise"],
                         t_offset=cfg["t_offset"])
    out = engine.autocorr(spec, n_traj, seed=0x5EED0001)
    return spec, out


def _check(case, out, n_traj):
    for key in ("fwd", "echo"):
        ref = np.array(case["columns"][key])
        a = out[key][0]
        mine = a.mean(axis=0)
        se = a.std(axis=0) / np.sqrt(n_traj)
        chi2, zmax = chi2_per_dof(ref, mine, shot_sigma(mine), se)
        assert chi2 < 2.0 and zmax < 4.5, (case["name"], key, chi2, zmax)


@pytest.mark.parametrize("name", ["L20_circ_x", "L20_circ_y", "L20_circ_circular_left",
                                  "L20_circ_circular_right", "L20_pol_x", "L20_pol_y",
                                  "L20_pol_xy", "L20_pol_yx", "L20_ctrl_standard_g97",
                                  "L20_ctrl_standard_g84"])
def test_L20_vs_reference_aer(pkg, engine, golden, name):
    case = [c for c in golden["aer_autocorr"] if c["name"] == name][0]
    _, out = _run_case(pkg, engine, golden, case)
    # t = 0 (and t = 1 echo) analytic values hold for every L
    p = case["config"]["noise"]
    if case["config"]["t_offset"] == 0:
        assert np.allclose(out["fwd"][0][:, 0], (1 - p) ** 6)
    _check(case, out, N_TRAJ)


@pytest.mark.parametrize("gain", ["0.01", "0.05"])
def test_L4_vs_reference_aer_and_exact(pkg, engine, golden, gain):
    case = _cases(golden, f"L4_ctrl_standard_gain{gain}")[0]
    n = 16384
    spec, out = _run_case(pkg, engine, golden, case, n)
    _check(case, out, n)
    f, e = dm_oracle.folded_sweep(4, spec.T, spec.hs[0], spec.phis[0], spec.kick, 0.05,
                                  t_offset=1)
    for key, exact in (("fwd", f), ("echo", e)):
        a = out[key][0]
        sd = a.std(axis=0)
        ok = sd > 1e-9
        z = np.abs(a.mean(axis=0) - exact)[ok] / (sd[ok] / np.sqrt(n))
        assert np.allclose(a.mean(axis=0)[~ok], exact[~ok], atol=1e-12)
        assert z.max() < 4.5


def test_config0_noiseless_L4_exact(pkg, engine, golden):
    """BASELINE configs[0]: L=4, g=0.97, tf=20, noiseless -> exact to 1e-10."""
    d = golden["disorder"]["L4"]
    spec = pkg.SweepSpec(L=4, T=20, hs=np.array(d["hs"]), phis=np.array(d["phis"]), g=0.97,
                         noise_prob=0.05, use_noise=0)
    out = engine.autocorr(spec, 1)
    from tests.test_oracle import KAT_FWD_P0

    np.testing.assert_allclose(out["fwd"][0, 0], KAT_FWD_P0, atol=1e-10)
    np.testing.assert_allclose(out["echo"][0, 0], np.ones(20), atol=1e-10)


def test_full_size_L20_properties(pkg, engine, golden):
    """At the bench configuration's full size: noiseless echo == 1 for every
    t (U^-t U^t = I), |<Z>| <= 1, norms preserved, and the t=1 analytic
    values under noise."""
    d = golden["disorder"]["L20"]
    hs, phis = np.array(d["hs"][:1]), np.array(d["phis"][:1])
    s0 = pkg.SweepSpec(L=20, T=30, hs=hs, phis=phis, g=0.97, noise_prob=0.0, use_noise=0)
    o0 = engine.autocorr(s0, 1)
    np.testing.assert_allclose(o0["echo"][0, 0], np.ones(30), atol=1e-10)
    assert np.all(np.abs(o0["fwd"]) <= 1 + 1e-12)
    s1 = pkg.SweepSpec(L=20, T=2, hs=hs, phis=phis, g=0.97, noise_prob=0.05)
    o1 = engine.autocorr(s1, 512, seed=3)
    p = 0.05
    e1 = o1["echo"][0][:, 1].mean()
    f1 = o1["fwd"][0][:, 1].mean()
    se = o1["echo"][0][:, 1].std() / np.sqrt(512)
    assert abs(e1 - (1 - p) ** 8) < 4.5 * se + 1e-12
    sf = o1["fwd"][0][:, 1].std() / np.sqrt(512)
    assert abs(f1 - (1 - p) ** 7 * np.cos(np.pi * 0.97)) < 4.5 * sf + 1e-12


def test_facade_runs_reference_shaped_circuits(pkg, golden):
    """AerSimulator-shaped facade on circuits built exactly like fast.py:124-147."""
    d = golden["disorder"]["L4"]
    hs, phis = d["hs"][0][:4], d["phis"][0][:3]
    nm = pkg.NoiseModel()
    nm.add_all_qubit_quantum_error(pkg.depolarizing_error(0.05, 1), ["u1", "u2", "u3"],
                                   warnings=False)
    backend = pkg.AerSimulator(noise_model=nm, device="GPU", cuStateVec_enable=True,
                               seed_simulator=5)
    kick = pkg.kick_table(4, 6, 0.97)
    f, e = dm_oracle.folded_sweep(4, 6, np.array(hs), np.array(phis), kick, 0.05)
    for t in (0, 3, 5):
        for echo in (False, True):
            circ = pkg.circuit.dtc_circuit(4, t, hs, phis, lambda s: [("rx", np.pi * 0.97)],
                                           echo=echo)
            ests = []
            for rep in range(8):
                counts = backend.run(circ, shots=1024).result().get_counts(circ)
                assert sum(counts.values()) == 1024
                ests.append(pkg.compute_z_expectation(counts, 1)[0])
            exact = (e if echo else f)[t]
            # 8 x 1024 shots: sigma ~ sqrt(1-A^2)/sqrt(8192)
            assert abs(np.mean(ests) - exact) < 4.5 * np.sqrt(1 - exact ** 2) / 90.5 + 1e-9
    # ideal circuit: one exact statevector, binomial shots
    ideal = pkg.AerSimulator(noise_model=None, seed_simulator=1)
    circ = pkg.circuit.dtc_circuit(4, 2, hs, phis, lambda s: [("rx", np.pi * 0.97)])
    res = ideal.run(circ, shots=4096).result()
    f0, _ = dm_oracle.folded_sweep(4, 3, np.array(hs), np.array(phis), kick, 0.0)
    assert abs(res.expectations[0] - f0[2]) < 1e-10
