"""Shared test helpers (random disorder, statistics)."""
import numpy as np


def random_disorder(rng, L, n_inst=1):
    hs = rng.uniform(-np.pi, np.pi, (n_inst, L))
    phis = rng.uniform(-1.5 * np.pi, -0.5 * np.pi, (n_inst, max(L - 1, 1)))
    return hs, phis


def shot_sigma(a, shots=1024):
    """Std of a (n0 - n1)/shots estimate with expectation a."""
    return np.sqrt(np.clip(1.0 - np.asarray(a) ** 2, 1e-4, None) / shots)


def chi2_per_dof(x, y, sx, sy):
    r = (np.asarray(x) - np.asarray(y)) / np.sqrt(np.asarray(sx) ** 2 + np.asarray(sy) ** 2)
    return float(np.mean(r ** 2)), float(np.max(np.abs(r)))


def harsh_device(pkg, L):
    """A device-like noise model with strong damping (the device tests')."""
    return pkg.DeviceNoise(p_gate=np.full(L, 0.02), t1_us=np.linspace(1.5, 3.0, L),
                           t2_us=np.linspace(1.0, 4.0, L), gate_ns=120.0, anc_factor=0.9,
                           readout_p01=0.02, readout_p10=0.035)
