"""Upper/lower envelopes of an autocorrelator series:
the ``*_env`` columns of the polarization scripts
(autocorr-delta-a-single-qiskit-fast-polarization.py:255-323, same in
-circular-polarization.py:277-345 and -xy-cycle) and of the controlled-g /
g-optimization scripts (-controlled-g.py:27-88, -g-optimization.py:27-88).

Algorithm (both variants):
  1. extrema: scipy.signal.find_peaks on +s and -s with distance
     max(1, window // 2); both end points are always added;
  2. interpolation of s at the extrema over all indices (interp1d with
     extrapolation) — polarization variant: cubic with >= 4 extrema, linear
     with 2-3; controlled variant: cubic with >= 2 (interp1d refuses fewer
     than 4 points for cubic, and the scripts then drop all envelope columns:
     ``EnvelopeUnavailable`` here);
  3. clamp (upper >= s, lower <= s), gaussian_filter1d with
     sigma = max(0.5, window / 4), clamp again.
Fewer than 2 extrema: the constant max(s) / min(s).
"""
from __future__ import annotations

import numpy as np


class EnvelopeUnavailable(ValueError):
    """The controlled-g variant's cubic interpolation had < 4 extrema."""


def _extrema(s: np.ndarray, window: int):
    from scipy.signal import find_peaks

    dist = max(1, window // 2)
    last = len(s) - 1
    out = []
    for sig in (s, -s):
        idx, _ = find_peaks(sig, distance=dist)
        idx = list(idx)
        if 0 not in idx:
            idx = [0] + idx
        if last not in idx:
            idx = idx + [last]
        out.append(np.sort(np.asarray(idx, dtype=np.int64)))
    return out


def _interp(s, idx, n, variant, fallback):
    from scipy.interpolate import interp1d

    if variant == "polarization":
        if len(idx) >= 4:
            kind = "cubic"
        elif len(idx) >= 2:
            kind = "linear"
        else:
            return np.full(n, fallback, dtype=float)
    else:
        if len(idx) < 2:
            return np.full(n, fallback, dtype=float)
        if len(idx) < 4:
            raise EnvelopeUnavailable("cubic envelope needs >= 4 extrema")
        kind = "cubic"
    f = interp1d(idx, s[idx], kind=kind, bounds_error=False, fill_value="extrapolate")
    return f(np.arange(n))


def find_envelope(signal, window_size: int = 5, variant: str = "polarization"):
    """Return ``(upper, lower)`` arrays like the reference's ``find_envelope``."""
    from scipy.ndimage import gaussian_filter1d

    if variant not in ("polarization", "controlled"):
        raise ValueError("variant must be 'polarization' or 'controlled'")
    s = np.asarray(signal, dtype=float)
    n = len(s)
    hi_idx, lo_idx = _extrema(s, window_size)
    upper = np.maximum(_interp(s, hi_idx, n, variant, np.max(s)), s)
    lower = np.minimum(_interp(s, lo_idx, n, variant, np.min(s)), s)
    sigma = max(0.5, window_size / 4)
    upper = np.maximum(gaussian_filter1d(upper, sigma=sigma), s)
    lower = np.minimum(gaussian_filter1d(lower, sigma=sigma), s)
    return upper, lower
