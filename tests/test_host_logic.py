"""Host-side logic (CPU): kick tables, disorder I/O, CSV schema, estimators,
circuit folding of reference-shaped circuits, sharding arithmetic."""
import math
import os

import numpy as np
import pytest

from oracle import dm_oracle
from tests.helpers import random_disorder


def test_rx_ry_match_qiskit_definitions(pkg):
    th = 0.97 * math.pi
    c, s = math.cos(th / 2), math.sin(th / 2)
    np.testing.assert_allclose(pkg.rx(th), [[c, -1j * s], [-1j * s, c]])
    np.testing.assert_allclose(pkg.ry(th), [[c, -s], [s, c]])
    for m in (pkg.rx(th), pkg.ry(0.3)):
        np.testing.assert_allclose(m @ m.conj().T, np.eye(2), atol=1e-15)


@pytest.mark.parametrize("pol,n_sub", [("x", 1), ("y", 1), ("xy", 2), ("yx", 2),
                                       ("circular_left", 2), ("circular_right", 2),
                                       ("circular_static", 2), ("xy_cycle", 1)])
def test_kick_table_shapes(pkg, pol, n_sub):
    tab = pkg.kick_table(5, 12, 0.9, pol)
    assert tab.shape == (12, 5, n_sub, 8)
    m = pkg.kicks.row_to_matrix(tab[3, 2, 0])
    np.testing.assert_allclose(m @ m.conj().T, np.eye(2), atol=1e-14)


def test_kick_table_semantics(pkg):
    g = 0.97
    # circular: angle_x = pi g cos(w s)/sqrt2, angle_y = +- pi g sin(w s)/sqrt2
    tl = pkg.kick_table(3, 4, g, "circular_left", circular_frequency=0.7)
    tr = pkg.kick_table(3, 4, g, "circular_right", circular_frequency=0.7)
    s = 2
    ax = math.pi * g * math.cos(0.7 * s) / math.sqrt(2)
    ay = math.pi * g * math.sin(0.7 * s) / math.sqrt(2)
    np.testing.assert_allclose(pkg.kicks.row_to_matrix(tl[s, 0, 0]), pkg.rx(ax))
    np.testing.assert_allclose(pkg.kicks.row_to_matrix(tl[s, 0, 1]), pkg.ry(ay))
    np.testing.assert_allclose(pkg.kicks.row_to_matrix(tr[s, 0, 1]), pkg.ry(-ay))
    # xy cycle: x for steps 0-4, y for 5-9
    tc = pkg.kick_table(2, 12, g, "xy_cycle")
    np.testing.assert_allclose(pkg.kicks.row_to_matrix(tc[4, 0, 0]), pkg.rx(math.pi * g))
    np.testing.assert_allclose(pkg.kicks.row_to_matrix(tc[5, 0, 0]), pkg.ry(math.pi * g))
    np.testing.assert_allclose(pkg.kicks.row_to_matrix(tc[10, 0, 0]), pkg.rx(math.pi * g))
    # per-period g list (controlled-g.py:215-227)
    gl = [0.84, 0.9, 0.95]
    tg = pkg.kick_table(2, 4, gl, "x")
    for s, gs in enumerate(gl + [0.84]):
        np.testing.assert_allclose(pkg.kicks.row_to_matrix(tg[s, 1, 0]), pkg.rx(math.pi * gs))


def test_neel_mask(pkg):
    # fast.py:127-130: X on circuit qubits 2,4,.. = sites 1,3,..
    assert pkg.init_mask(4, "vacuum") == 0
    assert pkg.init_mask(4, "neel") == 0b1010
    assert pkg.init_mask(5, "neel") == 0b01010
    with pytest.raises(ValueError):
        pkg.init_mask(4, "ghz")


def test_disorder_roundtrip(pkg, golden, tmp_path):
    import pandas as pd

    d = golden["disorder"]["L20"]
    hs = np.array(d["hs"])
    ph = np.array(d["phis"])
    pd.DataFrame(hs).to_csv(tmp_path / "hs_L20.csv", index=False,
                            header=[f"h_{i}" for i in range(20)])
    pd.DataFrame(ph).to_csv(tmp_path / "phis_L20.csv", index=False,
                            header=[f"phi_{i}" for i in range(19)])
    h2, p2 = pkg.load_disorder(20, 3, str(tmp_path))
    # pandas' default float parser (used by fast.py:71-72 too) is within 1 ulp
    np.testing.assert_allclose(h2, hs[:3], rtol=1e-15, atol=0)
    np.testing.assert_allclose(p2, ph[:3], rtol=1e-15, atol=0)
    # hs_L4.csv carries 6 columns (fast.py:66-74 slices implicitly); we take L / L-1
    d4 = golden["disorder"]["L4"]
    assert len(d4["hs"][0]) == 6 and len(d4["phis"][0]) == 5
    with pytest.raises(ValueError):
        pkg.load_disorder(20, 1000, str(tmp_path))
    # generator ranges (generate_disorder.py:16-20)
    h, p = pkg.generate_disorder(30, 50, seed=1)
    assert h.min() >= -math.pi and h.max() < math.pi
    assert p.min() >= -1.5 * math.pi and p.max() < -0.5 * math.pi
    hs_path, ph_path = pkg.save_disorder_to_csv(8, 4, folder=str(tmp_path), seed=2)
    assert os.path.basename(hs_path) == "hs_L8_inst4_ampl1.0_delta0.0_randomphi1.csv"
    assert list(pd.read_csv(ph_path).columns) == [f"phi_{i}" for i in range(7)]


def test_compute_z_expectation(pkg):
    f = pkg.compute_z_expectation
    assert f({"0": 700, "1": 324}, 1) == [(700 - 324) / 1024]
    assert f({"1": 1024}, 1) == [-1.0]
    assert f({"01": 3, "10": 1}, 2) == [(1 - 3) / 4, (3 - 1) / 4]


def test_autocorr_csv_schema(pkg, tmp_path):
    sw = pkg.sweep
    assert sw.folder_name(20, 0.05, 0) == "autocorr_data_L20_noiseprob0.05_fakebackend0"
    name = sw.autocorr_csv_name("vacuum", 0.97, 20, 1, 30, 1, 0.0, 1.0, 0.05, 1)
    assert name == ("autocorr_data_vacuum_g0.97_L20_inst1_tf30_randomphi1_delta0.0_"
                    "amplitude1.0_noise0.05_usenoise1.csv")
    path = sw.write_autocorr_csv(str(tmp_path / "x" / name), np.arange(3),
                                 np.array([0.7, -0.6, 0.5]), np.array([0.7, 0.25, -0.01]))
    import pandas as pd

    df = pd.read_csv(path)
    assert list(df.columns) == ["time", "av_autocorr", "av_autocorr_echo",
                                "sqrt_av_autocorr_echo"]
    assert df["sqrt_av_autocorr_echo"][1] == 0.5 and np.isnan(df["sqrt_av_autocorr_echo"][2])
    assert open(path).read().splitlines()[3].endswith(",")  # NaN written as empty


def test_shot_estimator_distribution(pkg):
    rng = np.random.default_rng(0)
    a = np.full((1, 1024, 3), 0.4)
    ests = np.array([pkg.sweep._shot_estimate(a, 1024, rng)[0] for _ in range(400)])
    assert abs(ests.mean() - 0.4) < 0.005
    assert abs(ests.std() - math.sqrt(1 - 0.16) / 32) < 0.004
    assert np.all(np.abs(ests * 512 - np.round(ests * 512)) < 1e-9)
    one = pkg.sweep._shot_estimate(np.full((2, 1, 4), -0.2), 1024, rng)
    assert one.shape == (2, 4)


def _ref_circuit(pkg, L, t, hs, phis, specs_fn, echo, state="vacuum"):
    return pkg.circuit.dtc_circuit(L, t, hs, phis, specs_fn, echo=echo, initial_state=state)


@pytest.mark.parametrize("pol", ["x", "xy", "circular_left", "xy_cycle"])
@pytest.mark.parametrize("echo", [False, True])
def test_fold_reference_circuits(pkg, pol, echo):
    rng = np.random.default_rng(1)
    L, t = 6, 7
    hs, phis = random_disorder(rng, L)
    specs = lambda s: pkg.kicks.period_gate_specs(pol, 0.93, s, 1.0)  # noqa: E731
    circ = _ref_circuit(pkg, L, t, hs[0], phis[0], specs, echo, "neel")
    nm = pkg.NoiseModel()
    nm.add_all_qubit_quantum_error(pkg.depolarizing_error(0.05, 1), ["u1", "u2", "u3"])
    f = pkg.aer.fold_circuit(circ, nm)
    assert (f.L, f.n_fwd, f.echo, f.probe) == (L, t, echo, 3)
    assert f.init_mask == pkg.init_mask(L, "neel")
    np.testing.assert_allclose(f.hs[0], hs[0])
    np.testing.assert_allclose(f.phis[0], phis[0])
    np.testing.assert_allclose(f.kick, pkg.kick_table(L, t, 0.93, pol), atol=1e-15)
    assert f.kick_noisy and f.n_anc_noisy == 6 and f.prep_noisy


def test_fold_matches_exact_density_matrix(pkg):
    """Folded problem -> exact folded DM == literal circuit DM (ties the
    facade's circuit analysis to the oracle)."""
    rng = np.random.default_rng(2)
    L, t = 4, 3
    hs, phis = random_disorder(rng, L)
    specs = lambda s: pkg.kicks.period_gate_specs("yx", 0.9, s)  # noqa: E731
    circ = _ref_circuit(pkg, L, t, hs[0], phis[0], specs, True)
    f = pkg.aer.fold_circuit(circ, None)
    fw, ec = dm_oracle.folded_sweep(L, t + 1, f.hs[0], f.phis[0], f.kick, 0.05)
    direct = dm_oracle.ancilla_circuit_expectation(L, t, hs[0], phis[0],
                                                   pkg.kick_table(L, t, 0.9, "yx"), 0.05,
                                                   echo=True)
    assert abs(ec[t] - direct) < 1e-12


def test_fold_rejects_other_circuits(pkg):
    qc = pkg.QuantumCircuit(3, 1)
    qc.h(0)
    qc.measure(0, 0)
    with pytest.raises(NotImplementedError):
        pkg.aer.fold_circuit(qc, None)
    rng = np.random.default_rng(3)
    hs, phis = random_disorder(rng, 4)
    circ = _ref_circuit(pkg, 4, 2, hs[0], phis[0], lambda s: [("rx", 1.0)], False)
    bad = pkg.QuantumCircuit(5, 1)
    for ins in circ.data[:-3]:
        bad.data.append(ins)
    bad.x(2)  # non-DTC gate inside the evolution
    for ins in circ.data[-3:]:
        bad.data.append(ins)
    with pytest.raises(NotImplementedError):
        pkg.aer.fold_circuit(bad, None)
    with pytest.raises(NotImplementedError):
        pkg.NoiseModel.from_backend(object())


def test_circuit_inverse_and_append(pkg):
    sub = pkg.QuantumCircuit(3)
    sub.rx(0.3, 1).rzz(0.2, 1, 2).rz(-0.1, 2)
    inv = sub.inverse()
    assert [(i.name, i.qubits, i.params) for i in inv.data] == [
        ("rz", (2,), (0.1,)), ("rzz", (1, 2), (-0.2,)), ("rx", (1,), (-0.3,))]
    qc = pkg.QuantumCircuit(4, 1)
    qc.append(sub, [0, 2, 3])
    assert qc.data[1].qubits == (2, 3)
    with pytest.raises(IndexError):
        qc.rx(0.1, 9)


def test_shard_range(pkg):
    sr = pkg.distributed.shard_range
    for n in (1, 7, 64, 1000):
        for w in (1, 2, 3, 8):
            blocks = [sr(n, w, r) for r in range(w)]
            assert blocks[0][0] == 0 and blocks[-1][1] == n
            for (a, b), (c, d) in zip(blocks, blocks[1:]):
                assert b == c
            assert max(b - a for a, b in blocks) - min(b - a for a, b in blocks) <= 1
