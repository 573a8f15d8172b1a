"""Exact numpy restatement of the reference circuit (density matrices).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as a checker; never by the product path.

Two independent restatements of autocorr-delta-a-single-qiskit-fast.py:

1. ``ancilla_circuit_expectation`` — the literal (L+1)-qubit circuit of
   ``qc_qiskit`` (fast.py:124-147) as Aer executes it after transpilation
   (fast.py:176-192): H -> u2, CZ(a, anc) -> u2.cx.u2 on the ancilla,
   RX -> u3, RY -> u3, X -> u3, RZZ -> cx.rz.cx, RZ -> rz, with
   ``depolarizing_error(p, 1)`` after every u1/u2/u3 (fast.py:84-86), and
   the Z expectation of the measured ancilla (fast.py:92-109).
2. ``folded_sweep`` — the L-qubit folding used by the engine:
   A(t) = (1-p)^6 Tr[Z_j E_t(rho0 Z_j)]  (SURVEY.md §0.6), for all t at once.

Both give exact expectations (no shot noise); tests check 1 == 2 to 1e-12,
and 2 against the known-answer tables and the reference's committed Aer CSVs
(statistically, tests/golden/).
"""
from __future__ import annotations

import math

import numpy as np

I2 = np.eye(2, dtype=np.complex128)
PX = np.array([[0, 1], [1, 0]], dtype=np.complex128)
PY = np.array([[0, -1j], [1j, 0]], dtype=np.complex128)
PZ = np.array([[1, 0], [0, -1]], dtype=np.complex128)
H = np.array([[1, 1], [1, -1]], dtype=np.complex128) / math.sqrt(2)


def rx(theta):
    c, s = math.cos(theta / 2), math.sin(theta / 2)
    return np.array([[c, -1j * s], [-1j * s, c]], dtype=np.complex128)


def ry(theta):
    c, s = math.cos(theta / 2), math.sin(theta / 2)
    return np.array([[c, -s], [s, c]], dtype=np.complex128)


class DM:
    """n-qubit operator (density matrix or Hermitian-conjugate-closed
    operator) with qubit q = bit q of the index (qiskit little-endian)."""

    def __init__(self, n: int, op: np.ndarray):
        self.n = n
        self.t = op.reshape((2,) * (2 * n)).astype(np.complex128)

    def _ax(self, q):
        return self.n - 1 - q

    def u1(self, q, U):
        a = self._ax(q)
        t = np.tensordot(U, self.t, axes=([1], [a]))
        t = np.moveaxis(t, 0, a)
        b = self.n + a
        t = np.tensordot(t, U.conj().T, axes=([b], [0]))
        self.t = np.moveaxis(t, -1, b)

    def diag(self, phase: np.ndarray):
        """rho <- D rho D^dagger for diagonal D = diag(phase) over the full index."""
        N = 1 << self.n
        m = self.t.reshape(N, N)
        m = phase[:, None] * m * phase.conj()[None, :]
        self.t = m.reshape((2,) * (2 * self.n))

    def depolarize(self, q, p):
        if p == 0.0:
            return
        base = self.t.copy()
        acc = (1 - 3 * p / 4) * base
        for P in (PX, PY, PZ):
            self.t = base.copy()
            self.u1(q, P)
            acc = acc + (p / 4) * self.t
        self.t = acc

    def kraus(self, q, ops):
        """rho <- sum_k K rho K^dagger on qubit q."""
        base = self.t.copy()
        acc = None
        for K in ops:
            self.t = base.copy()
            a = self._ax(q)
            t = np.tensordot(K, self.t, axes=([1], [a]))
            t = np.moveaxis(t, 0, a)
            b = self.n + a
            t = np.tensordot(t, K.conj().T, axes=([b], [0]))
            t = np.moveaxis(t, -1, b)
            acc = t if acc is None else acc + t
        self.t = acc

    def expect_z(self, q) -> complex:
        N = 1 << self.n
        m = self.t.reshape(N, N)
        x = np.arange(N)
        z = 1 - 2 * ((x >> q) & 1)
        return complex(np.sum(z * np.diag(m)))

    def matrix(self):
        N = 1 << self.n
        return self.t.reshape(N, N)

    def copy(self):
        d = DM.__new__(DM)
        d.n = self.n
        d.t = self.t.copy()
        return d


def _phase_rz(n, q, theta):
    x = np.arange(1 << n)
    z = 1 - 2 * ((x >> q) & 1)
    return np.exp(-0.5j * theta * z)


def _phase_rzz(n, a, b, theta):
    x = np.arange(1 << n)
    zz = (1 - 2 * ((x >> a) & 1)) * (1 - 2 * ((x >> b) & 1))
    return np.exp(-0.5j * theta * zz)


def device_channel(dm: DM, q: int, gamma: float, d: float, p: float):
    """Device-like noise after a kick sub-gate (include/dtc.h dtc_device_noise):
    amplitude damping gamma, dephasing Z w.p. d, depolarizing_error(p, 1)."""
    K0 = np.array([[1, 0], [0, math.sqrt(1 - gamma)]], dtype=np.complex128)
    K1 = np.array([[0, math.sqrt(gamma)], [0, 0]], dtype=np.complex128)
    dm.kraus(q, [K0, K1])
    dm.kraus(q, [math.sqrt(1 - d) * np.eye(2, dtype=np.complex128), math.sqrt(d) * PZ])
    dm.depolarize(q, p)


def _noise_after_kick(dm: DM, q: int, site: int, p):
    """p: depolarizing parameter, or a list of per-site (gamma, d, p) channels."""
    if isinstance(p, (list, tuple)):
        device_channel(dm, q, *p[site])
    else:
        dm.depolarize(q, p)


def _period(dm: DM, off: int, L: int, kick_gates, hs, phis, p, inverse=False):
    """One U_F (fast.py:111-121) on system qubits off..off+L-1, or its inverse
    (fast.py:140-143).  ``kick_gates[i]`` = sub-gate list of site i; ``p`` =
    depolarizing parameter or per-site device channels (device_channel)."""
    n = dm.n
    if not inverse:
        for i in range(L):
            for G in kick_gates[i]:
                dm.u1(off + i, G)
                _noise_after_kick(dm, off + i, i, p)
        for i in list(range(0, L - 1, 2)) + list(range(1, L - 1, 2)):
            dm.diag(_phase_rzz(n, off + i, off + i + 1, phis[i]))
        for i in range(L):
            dm.diag(_phase_rz(n, off + i, hs[i]))
    else:
        for i in reversed(range(L)):
            dm.diag(_phase_rz(n, off + i, -hs[i]))
        for i in reversed(list(range(0, L - 1, 2)) + list(range(1, L - 1, 2))):
            dm.diag(_phase_rzz(n, off + i, off + i + 1, -phis[i]))
        for i in reversed(range(L)):
            for G in reversed(kick_gates[i]):
                dm.u1(off + i, G.conj().T)
                _noise_after_kick(dm, off + i, i, p)


def kick_gates_from_table(kick_row: np.ndarray):
    """[L][n_sub][8] ABI row -> per-site list of 2x2 matrices."""
    out = []
    for i in range(kick_row.shape[0]):
        gates = []
        for q in range(kick_row.shape[1]):
            r = kick_row[i, q].reshape(4, 2)
            gates.append((r[:, 0] + 1j * r[:, 1]).reshape(2, 2))
        out.append(gates)
    return out


def ancilla_circuit_expectation(L, t, hs, phis, kick, p, echo=False, initial_state="vacuum",
                                probe=None, t_offset=0):
    """<Z_ancilla> of the literal transpiled circuit for ONE time point t
    (fast.py:124-147).  ``kick``: [n_periods][L][n_sub][8] table."""
    j = int(L / 2) if probe is None else probe
    n = L + 1
    rho0 = np.zeros((1 << n, 1 << n), dtype=np.complex128)
    rho0[0, 0] = 1
    dm = DM(n, rho0)
    if initial_state == "neel":
        for q in range(1, L + 1):
            if q % 2 == 0:
                dm.u1(q, PX)          # x -> u3(pi, 0, pi): noisy
                dm.depolarize(q, p)
    dm.u1(0, H)                       # h -> u2: noisy
    dm.depolarize(0, p)

    def cz():
        # CZ(j+1, 0) -> u2(anc) . cx(j+1 -> anc) . u2(anc)
        dm.u1(0, H)
        dm.depolarize(0, p)
        N = 1 << n
        x = np.arange(N)
        perm = np.where((x >> (j + 1)) & 1, x ^ 1, x)
        m = dm.matrix()[perm][:, perm]
        dm.t = m.reshape((2,) * (2 * n))
        dm.u1(0, H)
        dm.depolarize(0, p)

    cz()
    n_per = t + t_offset
    for s in range(n_per):
        _period(dm, 1, L, kick_gates_from_table(kick[s]), hs, phis, p)
    if echo:
        for s in reversed(range(n_per)):
            _period(dm, 1, L, kick_gates_from_table(kick[s]), hs, phis, p, inverse=True)
    cz()
    dm.u1(0, H)
    dm.depolarize(0, p)
    return dm.expect_z(0).real


def folded_sweep(L, T, hs, phis, kick, p, initial_state="vacuum", probe=None, t_offset=0,
                 n_anc=6, want_echo=True):
    """Exact A_fwd(t), A_echo(t) for t = 0..T-1 with the L-qubit folding."""
    j = int(L / 2) if probe is None else probe
    N = 1 << L
    # rho0: neel X gates followed by depolarizing draws (X/Y undo the flip)
    probs = []
    for i in range(L):
        q = i + 1
        flipped = initial_state == "neel" and q % 2 == 0
        probs.append((1 - p / 2) if flipped else 0.0)
    x = np.arange(N)
    w = np.ones(N)
    for i, pf in enumerate(probs):
        b = (x >> i) & 1
        w = w * np.where(b == 1, pf, 1 - pf)
    zj = 1 - 2 * ((x >> j) & 1)
    sigma = DM(L, np.diag(w * zj).astype(np.complex128))
    fac = (1 - p) ** n_anc
    fwd = np.zeros(T)
    echo = np.zeros(T)
    for s in range(T - 1 + t_offset + 1):
        if s > 0:
            _period(sigma, 0, L, kick_gates_from_table(kick[s - 1]), hs, phis, p)
        t = s - t_offset
        if t < 0:
            continue
        fwd[t] = fac * sigma.expect_z(j).real
        if want_echo:
            e = sigma.copy()
            for k in range(s, 0, -1):
                _period(e, 0, L, kick_gates_from_table(kick[k - 1]), hs, phis, p, inverse=True)
            echo[t] = fac * e.expect_z(j).real
    return fwd, echo


def device_folded_sweep(L, T, hs, phis, kick, dev, initial_state="vacuum", probe=None,
                        t_offset=0, want_echo=True):
    """Exact read-out A_fwd(t), A_echo(t) under device-like noise (``dev`` a
    DeviceNoise): the folded L-qubit model with the per-site channel after
    every kick sub-gate, the neel-prep X followed by its Pauli part only,
    then anc_factor and the ancilla read-out map (include/dtc.h)."""
    j = int(L / 2) if probe is None else probe
    N = 1 << L
    ch = dev.site_channels()
    x = np.arange(N)
    w = np.ones(N)
    for i in range(L):
        flipped = initial_state == "neel" and (i + 1) % 2 == 0
        pf = (1 - ch[i][2] / 2) if flipped else 0.0   # X/Y after X undo the flip
        b = (x >> i) & 1
        w = w * np.where(b == 1, pf, 1 - pf)
    zj = 1 - 2 * ((x >> j) & 1)
    sigma = DM(L, np.diag(w * zj).astype(np.complex128))
    fwd = np.zeros(T)
    echo = np.zeros(T)
    for s in range(T - 1 + t_offset + 1):
        if s > 0:
            _period(sigma, 0, L, kick_gates_from_table(kick[s - 1]), hs, phis, ch)
        t = s - t_offset
        if t < 0:
            continue
        fwd[t] = dev.readout(dev.anc_factor * sigma.expect_z(j).real)
        if want_echo:
            e = sigma.copy()
            for k in range(s, 0, -1):
                _period(e, 0, L, kick_gates_from_table(kick[k - 1]), hs, phis, ch, inverse=True)
            echo[t] = dev.readout(dev.anc_factor * e.expect_z(j).real)
    return fwd, echo


def statevector_zsite(L, T, hs, phis, kick, init_mask=0, t_offset=0):
    """Noiseless statevector <Z_i>(t), t = 0..T-1 (L up to ~20)."""
    N = 1 << L
    psi = np.zeros(N, dtype=np.complex128)
    psi[init_mask] = 1
    x = np.arange(N)
    z = 1 - 2 * ((x[None, :] >> np.arange(L)[:, None]) & 1)
    ang = np.zeros(N)
    for i in range(L):
        ang += hs[i] * z[i]
    for i in range(L - 1):
        ang += phis[i] * z[i] * z[i + 1]
    diag = np.exp(-0.5j * ang)
    out = np.zeros((T, L))
    for s in range(T - 1 + t_offset + 1):
        if s > 0:
            gates = kick_gates_from_table(kick[s - 1])
            psi = psi.reshape((2,) * L)
            for i in range(L):
                ax = L - 1 - i
                for G in gates[i]:
                    psi = np.moveaxis(np.tensordot(G, psi, axes=([1], [ax])), 0, ax)
            psi = psi.reshape(N) * diag
        t = s - t_offset
        if t >= 0:
            pr = np.abs(psi) ** 2
            out[t] = z @ pr
    return out


def energy_sweep(L, T, hs, phis, kick, p, initial_state="vacuum", t_offset=0, dev=None):
    """Exact <Z_i>, <Z_i Z_i+1>, <X_i> of the L-qubit energy circuit
    (autocorr-delta-a-single-qiskit-fast-energy.py:136-150: optional neel X
    gates on qubits 2, 4, .., L-1 (even L raises, as qiskit does), then t periods of fast.py's U_F, no ancilla) under the depolarizing
    channel after every kick gate and prep X, for t = 0..T-1.  ``dev`` (a
    DeviceNoise): the device-like channel instead (p unused), no read-out."""
    N = 1 << L
    x = np.arange(N)
    w = np.ones(N)
    if dev is not None:
        p = dev.site_channels()
    # neel (energy.py:138-141): X on qubit i for i in 1..L with i even, on an
    # L-qubit circuit whose qubit i is site i; i = L (even L) is out of range
    neel = set()
    if initial_state == "neel":
        for i in range(1, L + 1):
            if i % 2 == 0:
                if i >= L:
                    raise ValueError("neel on an even-L energy circuit: qubit L out of range")
                neel.add(i)
    for i in range(L):
        flipped = i in neel
        pi = p[i][2] if dev is not None else p
        pf = (1 - pi / 2) if flipped else 0.0
        b = (x >> i) & 1
        w = w * np.where(b == 1, pf, 1 - pf)
    rho = DM(L, np.diag(w).astype(np.complex128))
    z = np.zeros((T, L))
    zz = np.zeros((T, max(L - 1, 0)))
    xs = np.zeros((T, L))
    zbits = 1 - 2 * ((x[None, :] >> np.arange(L)[:, None]) & 1)
    for s in range(T - 1 + t_offset + 1):
        if s > 0:
            _period(rho, 0, L, kick_gates_from_table(kick[s - 1]), hs, phis, p)
        t = s - t_offset
        if t < 0:
            continue
        m = rho.matrix()
        d = np.real(np.diag(m))
        z[t] = zbits @ d
        for i in range(L - 1):
            zz[t, i] = (zbits[i] * zbits[i + 1]) @ d
        for i in range(L):
            # <X_i> = 2 Re sum_{x: bit i = 0} rho[x ^ e_i, x]
            lo = x[((x >> i) & 1) == 0]
            xs[t, i] = 2.0 * np.real(m[lo ^ (1 << i), lo]).sum()
    return z, zz, xs
