"""Energy path host logic and oracles (no GPU): the big-endian Hamiltonian
labels of energy.py:83-102 vs the little-endian coefficients the engine's
observables are combined with; exact density-matrix energies vs the
per-trajectory oracle; the accumulated-noise loop (energy.py:212-218)."""
import numpy as np
import pytest

from oracle import dm_oracle, energy_oracle
from tests.helpers import random_disorder

I2 = np.eye(2)
PAULI = {"I": I2, "X": np.array([[0, 1], [1, 0]]), "Z": np.diag([1.0, -1.0])}


def _label_matrix(label):
    # qiskit: label[0] is the highest qubit -> leftmost Kronecker factor
    m = np.array([[1.0]])
    for ch in label:
        m = np.kron(m, PAULI[ch])
    return m


def _site_op(L, q, P):
    m = np.array([[1.0]])
    for k in reversed(range(L)):  # bit q of the index = qubit q
        m = np.kron(m, P if k == q else I2)
    return m


@pytest.mark.parametrize("L", [3, 4, 5])
@pytest.mark.parametrize("ht", ["full", "z_only", "zz_only", "x_only", "z_zz"])
def test_big_endian_labels_match_coefficients(pkg, L, ht):
    rng = np.random.default_rng(L)
    hs, phis = random_disorder(rng, L)
    g = 0.93
    H_ref = sum(c * _label_matrix(lab)
                for lab, c in pkg.energy.hamiltonian_labels(L, g, hs[0], phis[0], ht))
    cz, czz, cx = pkg.energy.hamiltonian_coefficients(L, g, hs[0], phis[0], ht)
    H = np.zeros((1 << L, 1 << L))
    for q in range(L):
        H += cz[q] * _site_op(L, q, PAULI["Z"]) + cx[q] * _site_op(L, q, PAULI["X"])
    for q in range(L - 1):
        H += czz[q] * _site_op(L, q, PAULI["Z"]) @ _site_op(L, q + 1, PAULI["Z"])
    assert np.abs(H - H_ref).max() < 1e-12
    if ht in ("full", "z_only"):
        assert cz[L - 1] == hs[0][0]  # reversed w.r.t. the circuit's RZ(hs[i]) on qubit i


def test_accumulated_noise(pkg):
    eff = pkg.energy.accumulated_noise([0, 0.001, 0.01, 0.1])
    assert eff[0] == 0.0
    assert abs(eff[1] - 0.001) < 1e-15
    assert abs(eff[2] - (1 - 0.999 * 0.99)) < 1e-15
    assert abs(eff[3] - (1 - 0.999 * 0.99 * 0.9)) < 1e-15


def test_trajectory_oracle_noiseless_equals_dm(pkg):
    rng = np.random.default_rng(2)
    L, T = 5, 6
    hs, phis = random_disorder(rng, L)
    spec = pkg.energy.energy_spec(L, T, hs, phis, 0.9, "neel", use_noise=0, polarization="xy")
    z, zz, x = energy_oracle.trajectory_energy(spec, 0, 0)
    dz, dzz, dx = dm_oracle.energy_sweep(L, T, hs[0], phis[0], spec.kick, 0.0, "neel")
    assert np.abs(z - dz).max() < 1e-12
    assert np.abs(zz - dzz).max() < 1e-12
    assert np.abs(x - dx).max() < 1e-12


def test_trajectory_mean_converges_to_dm(pkg):
    rng = np.random.default_rng(3)
    L, T, p, n = 5, 5, 0.1, 600
    hs, phis = random_disorder(rng, L)
    spec = pkg.energy.energy_spec(L, T, hs, phis, 0.95, "neel", noise_prob=p)
    acc = [np.zeros((T, L)), np.zeros((T, L - 1)), np.zeros((T, L))]
    sq = [np.zeros_like(a) for a in acc]
    for tr in range(n):
        for k, v in enumerate(energy_oracle.trajectory_energy(spec, 0, tr, seed=11)):
            acc[k] += v
            sq[k] += v * v
    exact = dm_oracle.energy_sweep(L, T, hs[0], phis[0], spec.kick, p, "neel")
    for k in range(3):
        mean = acc[k] / n
        sd = np.sqrt(np.maximum(sq[k] / n - mean ** 2, 0) / n)
        r = np.abs(mean - exact[k])
        assert np.all((r < 5 * sd + 1e-12)), (k, r.max())


def test_energy_decomposition(pkg):
    rng = np.random.default_rng(4)
    L, T = 4, 3
    hs, phis = random_disorder(rng, L)
    obs = {"z": rng.normal(size=(T, L)), "zz": rng.normal(size=(T, L - 1)),
           "x": rng.normal(size=(T, L))}
    e = {ht: pkg.energy.energy_from_observables(obs, L, 0.97, hs[0], phis[0], ht)
         for ht in pkg.energy.HAMILTONIAN_TYPES}
    assert np.allclose(e["full"], e["z_only"] + e["zz_only"] + e["x_only"])
    assert np.allclose(e["z_zz"], e["z_only"] + e["zz_only"])


def test_energy_neel_mapping(pkg):
    """energy.py:138-141 on QuantumCircuit(L): X on qubits 2, 4, ..., L-1 (qubit i is
    site i, no ancilla) -- not the autocorrelator's ancilla-offset sites 1, 3, ..."""
    def literal(L):
        flips = []
        for i in range(1, L + 1):       # the reference's loop, restated
            if i % 2 == 0:
                if not i < L:           # QuantumCircuit(L).x(i) needs 0 <= i < L
                    raise IndexError(i)
                flips.append(i)
        return sum(1 << i for i in flips)

    for L in (1, 3, 5, 7, 9, 21):
        assert pkg.energy_init_mask(L, "neel") == literal(L)
    assert pkg.energy_init_mask(5, "neel") == 0b10100
    assert pkg.energy_init_mask(7, "neel") == 0b1010100
    assert pkg.init_mask(5, "neel") == 0b01010    # the ancilla circuit's mapping
    assert pkg.energy_init_mask(6, "vacuum") == 0


@pytest.mark.parametrize("L", [2, 4, 6, 20])
def test_energy_neel_even_L_rejected(pkg, L):
    """For even L the reference's circ.x(L) is out of range and raises; the
    energy path and its oracle refuse the same inputs."""
    rng = np.random.default_rng(L)
    hs, phis = random_disorder(rng, L)
    with pytest.raises(ValueError, match="out of range"):
        pkg.energy.energy_spec(L, 3, hs, phis, 0.97, "neel")
    with pytest.raises(ValueError):
        pkg.energy.run_energy(L, 0.97, hs, phis, 3, initial_state="neel", engine=object())
    with pytest.raises(ValueError):
        dm_oracle.energy_sweep(L, 3, hs[0], phis[0], np.zeros((2, L, 1, 8)), 0.0, "neel")


def test_energy_neel_odd_L_exact(pkg):
    """Noiseless neel t=0 values of the energy circuit: Z_i = -1 on sites 2, 4, .."""
    rng = np.random.default_rng(11)
    L = 7
    hs, phis = random_disorder(rng, L)
    spec = pkg.energy.energy_spec(L, 2, hs, phis, 0.9, "neel", use_noise=0)
    z, zz, x = dm_oracle.energy_sweep(L, 2, hs[0], phis[0], spec.kick, 0.0, "neel")
    assert list(z[0]) == [1, 1, -1, 1, -1, 1, -1]
