"""The Pauli-frame records of the 13-site pass (dtc_kernels.hip
frame13_records, dtc_tile13.hip), restated in numpy and checked against the
direct products of the kicks (CPU, test infrastructure).

The 13-site K-D-K pass runs one butterfly for every kick -- the form-B one,
G(f) = f I + i X (RX family) or f I + i Y (RY) -- with the kick's other forms
carried as a Pauli frame: form A is -i X G(-beta) (RX) or X Z G(-beta) (RY),
sigma = -1 a Z after the kick.  The frame's X bits are flushed by the pass's
re-layouts (the tile is permuted by X^m), its Z bits by the diagonal (a sign
per amplitude).  This model applies a pass's 26 kicks (random rotations of the
family times random Paulis and phases, canonicalised as the prep kernel does)
both ways on a 13-qubit state and requires the same state to rounding: the
algebra the kernels implement.  The GPU tests (test_gpu_split13.py) check the
kernels themselves against the oracle (autocorr-delta-a-single-qiskit-fast.py
:111-121, the Floquet period; :140-147, the echo)."""
import numpy as np
import pytest

NB = 13
X = np.array([[0, 1], [1, 0]], dtype=complex)
Y = np.array([[0, -1j], [1j, 0]], dtype=complex)
Z = np.diag([1.0 + 0j, -1.0])
PAULI = [np.eye(2, dtype=complex), X, Y, Z]


def rot(kind, t):
    c, s = np.cos(t / 2), np.sin(t / 2)
    if kind == "rx":
        return np.array([[c, -1j * s], [-1j * s, c]])
    return np.array([[c, -s], [s, c]], dtype=complex)


def canonicalise(kind, m):
    """dtc_kernels.hip canonicalise (unitary RX / RY families)."""
    if kind == "rx":
        a_form = m[0, 0].imag == 0 and m[0, 1].real == 0 and m[1, 0].real == 0 and m[1, 1].imag == 0
        a = m[0, 0].real if a_form else m[0, 0].imag
        b = m[0, 1].imag if a_form else -m[0, 1].real
        c = m[1, 0].imag if a_form else -m[1, 0].real
        d = m[1, 1].real if a_form else m[1, 1].imag
        k, sg = (0 if a_form else 1), a * d + b * c
    else:
        real = not np.any(m.imag)
        a, b, c, d = (x.real if real else x.imag for x in (m[0, 0], m[0, 1], m[1, 0], m[1, 1]))
        k, sg = (0 if real else 1), a * d - b * c
    form_b = abs(a) < abs(b)
    return dict(k=k, var=(2 if form_b else 0) | (1 if sg < 0 else 0),
                scale=b if form_b else a, coef=a / b if form_b else b / a)


def frame13(kind, recs):
    """frame13_records: recs[h][q] (h = pre / post, q = tile bit).  Returns the
    signed coefficients f[h][q], the masks (x1, x2, z, x3, x4) and the extra
    power of i."""
    rx = kind == "rx"
    x = z = ph = 0
    f = [[0.0] * NB for _ in range(2)]

    def form_a(r):
        return (r["var"] >> 1) ^ 1

    def zbit(r):
        return (r["var"] & 1) if rx else ((r["var"] & 1) ^ form_a(r))

    def kick(h, q):
        nonlocal x, z, ph
        r = recs[h][q]
        fa, n2 = form_a(r), zbit(r)
        g = -r["coef"] if fa else r["coef"]
        flip = ((z if rx else x ^ z) >> q) & 1
        f[h][q] = -g if flip else g
        ph += (3 * fa if rx else 2 * fa) + 2 * flip
        x ^= fa << q
        ph += 2 * (n2 & (x >> q) & 1)
        z ^= n2 << q

    def flush(m):
        nonlocal x, ph
        ph += 2 * (bin(z & m).count("1") & 1)
        x ^= m
        return m

    def xbits(h, q0, q1):
        return sum(form_a(recs[h][q]) << q for q in range(q0, q1 + 1))

    for q in range(4, 9):
        kick(0, q)
    m1 = flush(x)
    for q in range(4):
        kick(0, q)
    m2 = flush(x ^ xbits(0, 9, 12))
    for q in range(9, 13):
        kick(0, q)
    md = z ^ sum(zbit(recs[1][q]) << q for q in range(NB))
    z ^= md
    for q in range(9, 13):
        kick(1, q)
    m3 = flush(x)
    for q in range(4):
        kick(1, q)
    m4 = flush(x ^ xbits(1, 4, 8))
    for q in (8, 4, 5, 6, 7):
        kick(1, q)
    assert x == 0 and z == 0
    return f, (m1, m2, md, m3, m4), ph


def apply1(psi, q, m):
    s = psi.reshape(-1, 2, 1 << q)
    return np.einsum("ij,ajb->aib", m, s).reshape(-1)


def butterfly(kind, f):
    return np.array([[f, 1j], [1j, f]]) if kind == "rx" else np.array([[f, 1], [-1, f]], dtype=complex)


IDX = np.arange(1 << NB)
PAR = np.array([bin(i).count("1") & 1 for i in range(1 << 16)])


def xperm(v, m):
    return v[IDX ^ m]


def zsign(v, m):
    return v * np.where(PAR[IDX & m], -1.0, 1.0)


@pytest.mark.parametrize("kind", ["rx", "ry"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_frame13_matches_direct_kicks(kind, seed):
    rng = np.random.default_rng(seed)
    th = rng.uniform(0, 2 * np.pi)
    mats = [[None] * NB for _ in range(2)]
    for h in range(2):
        for q in range(NB):
            m = rot(kind, th if rng.random() < 0.6 else rng.uniform(-7, 7))
            m = PAULI[rng.integers(4)] @ m
            if rng.random() < 0.2:
                m = m * 1j ** rng.integers(4)
            if rng.random() < 0.05:
                m = np.eye(2, dtype=complex)  # a skipped site: the identity record
            m = np.where(np.abs(m.real) < 1e-15, 1j * m.imag, m)
            mats[h][q] = np.where(np.abs(m.imag) < 1e-15, m.real + 0j, m)
    recs = [[canonicalise(kind, mats[h][q]) for q in range(NB)] for h in range(2)]
    diag = np.exp(1j * rng.uniform(0, 2 * np.pi, 1 << NB))
    psi = rng.normal(size=1 << NB) + 1j * rng.normal(size=1 << NB)
    ref = psi.copy()
    for q in range(NB):
        ref = apply1(ref, q, mats[0][q])
    ref = ref * diag
    for q in range(NB):
        ref = apply1(ref, q, mats[1][q])

    f, (m1, m2, md, m3, m4), ph = frame13(kind, recs)
    ksum = sum(r["k"] for h in range(2) for r in recs[h])
    gph = 1j ** ((ksum + ph) % 4) * np.prod([r["scale"] for h in range(2) for r in recs[h]])
    v = psi.copy()
    for q in (4, 5, 6, 7, 8):
        v = apply1(v, q, butterfly(kind, f[0][q]))
    v = xperm(v, m1)
    for q in range(4):
        v = apply1(v, q, butterfly(kind, f[0][q]))
    v = xperm(v, m2)
    for q in range(9, 13):
        v = apply1(v, q, butterfly(kind, f[0][q]))
    v = zsign(v * diag * gph, md)
    for q in range(9, 13):
        v = apply1(v, q, butterfly(kind, f[1][q]))
    v = xperm(v, m3)
    for q in range(4):
        v = apply1(v, q, butterfly(kind, f[1][q]))
    v = xperm(v, m4)
    for q in (8, 4, 5, 6, 7):
        v = apply1(v, q, butterfly(kind, f[1][q]))
    assert np.abs(v - ref).max() < 1e-12 * np.abs(ref).max()
    # every coefficient the kernel multiplies by is at most 1 in magnitude
    assert max(abs(c) for row in f for c in row) <= 1.0 + 1e-15
