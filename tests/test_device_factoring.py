"""The factorisation the device-noise kernels rely on (SiteMat in
csrc/dtc_kernels.hip, kKindRXU / kKindRYU): every one-sub-gate device-like kick
Kraus x Pauli x RX(theta) (or RY) equals i^k * w * diag(rho0, rho1) * S, with S
the unitary-family butterfly of form A ([[1, i beta], [i beta, 1]]) or form B
([[alpha, i], [i, alpha]]) (RY: [[1, beta], [-beta, 1]] / [[alpha, 1], [-1, alpha]]),
so the kernels run S and defer the real diagonal.  Pure numpy restatement of the
canonicalisation (no GPU): the reconstruction must equal the kick to rounding,
including the jump operator followed by X or Y (a zero first row: rho0 = 0).
"""
import numpy as np
import pytest

X = np.array([[0, 1], [1, 0]], complex)
Y = np.array([[0, -1j], [1j, 0]])
Z = np.diag([1.0, -1.0]).astype(complex)
I2 = np.eye(2, dtype=complex)


def rx(th):
    c, s = np.cos(th / 2), np.sin(th / 2)
    return np.array([[c, -1j * s], [-1j * s, c]])


def ry(th):
    c, s = np.cos(th / 2), np.sin(th / 2)
    return np.array([[c, -s], [s, c]], complex)


def canonicalise(kind, m):
    """(k, w, rho0, rho1, coef, form_b) as the prep kernel computes them."""
    m = m.flatten()
    if kind == "rx":
        a_form = m[0].imag == 0 and m[1].real == 0 and m[2].real == 0 and m[3].imag == 0
        a = m[0].real if a_form else m[0].imag
        b = m[1].imag if a_form else -m[1].real
        c = m[2].imag if a_form else -m[2].real
        d = m[3].real if a_form else m[3].imag
        k = 0 if a_form else 1
    else:
        real = all(x.imag == 0 for x in m)
        a, b, c, d = [(x.real if real else x.imag) for x in m]
        k = 0 if real else 1
    is_rx = kind == "rx"
    if a != 0 or b != 0:
        form_b = abs(a) < abs(b)
        w = b if form_b else a
        coef = a / b if form_b else b / a
        rho0 = 1.0
        rho1 = ((c / b if is_rx else -c / b) if form_b else d / a)
    elif c != 0 or d != 0:
        form_b = abs(d) < abs(c)
        w = (c if is_rx else -c) if form_b else d
        coef = d / w if form_b else (c / d if is_rx else -c / d)
        rho0, rho1 = 0.0, 1.0
    else:
        return k, 0.0, 0.0, 0.0, 0.0, False
    return k, w, rho0, rho1, coef, form_b


def rebuild(kind, k, w, rho0, rho1, coef, form_b):
    if kind == "rx":
        s = np.array([[coef, 1j], [1j, coef]]) if form_b else np.array([[1, 1j * coef], [1j * coef, 1]])
    else:
        s = np.array([[coef, 1], [-1, coef]], complex) if form_b else np.array([[1, coef], [-coef, 1]], complex)
    return (1j ** k) * w * np.diag([rho0, rho1]) @ s


@pytest.mark.parametrize("kind", ["rx", "ry"])
def test_device_kick_factorisation(kind):
    rng = np.random.default_rng(7)
    gate = rx if kind == "rx" else ry
    worst = 0.0
    zero_first_rows = 0
    for _ in range(4000):
        g = gate(rng.uniform(0, 2 * np.pi))
        if rng.random() < 0.5:
            g = g.conj().T  # inverse kicks (the echo)
        k0, k1, kj = rng.uniform(0.3, 1.5, 3)
        kraus = np.diag([k0, k1]) if rng.random() < 0.5 else np.array([[0, kj], [0, 0]])
        p = [I2, X, Y, Z][rng.integers(4)]
        m = p @ kraus @ g
        parts = canonicalise(kind, m)
        zero_first_rows += parts[2] == 0.0 and parts[1] != 0.0
        worst = max(worst, float(np.abs(rebuild(kind, *parts) - m).max()))
    assert worst < 1e-14
    assert zero_first_rows > 100  # the jump followed by X or Y is exercised


def test_unitary_kicks_have_sign_rho():
    """Without a Kraus factor rho0 = 1 and rho1 = sigma = +-1 (the unitary
    family's source-negate variant)."""
    rng = np.random.default_rng(3)
    for _ in range(500):
        m = [I2, X, Y, Z][rng.integers(4)] @ rx(rng.uniform(0, 2 * np.pi))
        _, _, rho0, rho1, _, _ = canonicalise("rx", m)
        assert rho0 == 1.0 and abs(abs(rho1) - 1.0) < 1e-12
