"""Per-trajectory energy observables (TEST INFRASTRUCTURE ONLY: imported by
tests/, never by the product).

Follows one noisy trajectory of the L-qubit energy circuit
(autocorr-delta-a-single-qiskit-fast-energy.py:136-150) with the C oracle's
gate-by-gate periods (oracle/dtc_oracle.c via c_oracle.apply_periods, same
Philox draws as the engine: forward stream 0, period counter = period) and
evaluates <Z_i>, <Z_i Z_i+1>, <X_i> of the state after every period in numpy.
Under device-like noise (spec.device) the periods are the C oracle's
Kraus-weighted ones and the observables are the unnormalised (weighted)
expectations, before any read-out error.
"""
from __future__ import annotations

import numpy as np

from . import c_oracle

STREAM_PREP = 0xFFFFFFFF


def prep_mask(spec, seed, traj):
    """Noisy neel preparation (X then a Pauli draw: X/Y undo the flip; under
    device-like noise the draw of the C oracle's composite channel)."""
    if getattr(spec, "device", None) is not None:
        return c_oracle.init_mask(spec, seed, traj)
    m = spec.init_mask
    if spec.p > 0:
        for i in range(spec.L):
            if (spec.init_mask >> i) & 1:
                if c_oracle.sample_pauli(spec.p, seed, traj, STREAM_PREP, 0, i, 0) in (1, 2):
                    m &= ~(1 << i)
    return m


def observables(psi, L):
    """<Z_i>, <Z_i Z_i+1>, <X_i> of a state vector (one site at a time, so
    L=24 stays within a few hundred MB)."""
    x = np.arange(1 << L, dtype=np.int64)
    pr = np.abs(psi) ** 2
    zsign = [1.0 - 2.0 * ((x >> i) & 1) for i in range(L)]
    z = np.array([zb @ pr for zb in zsign])
    zz = np.array([(zsign[i] * zsign[i + 1]) @ pr for i in range(L - 1)])
    xs = np.empty(L)
    for i in range(L):
        lo = x[((x >> i) & 1) == 0]
        xs[i] = 2.0 * np.real(np.conj(psi[lo]) * psi[lo ^ (1 << i)]).sum()
    return z, zz, xs


def trajectory_energy(spec, inst, traj, seed=0x5EED0001):
    """z [T][L], zz [T][L-1], x [T][L] of one trajectory of instance ``inst``."""
    import dataclasses

    one = dataclasses.replace(spec, hs=spec.hs[inst:inst + 1], phis=spec.phis[inst:inst + 1])
    L, T = spec.L, spec.T
    psi = np.zeros(1 << L, dtype=np.complex128)
    psi[prep_mask(spec, seed, traj)] = 1.0
    z = np.zeros((T, L))
    zz = np.zeros((T, max(L - 1, 0)))
    xs = np.zeros((T, L))
    for s in range(T - 1 + spec.t_offset + 1):
        if s > 0:
            psi, _ = c_oracle.apply_periods(one, psi, s, 1, inst=0, traj=traj, stream=0,
                                            seed=seed)
        t = s - spec.t_offset
        if t >= 0:
            z[t], zz[t], xs[t] = observables(psi, L)
    return z, zz, xs
