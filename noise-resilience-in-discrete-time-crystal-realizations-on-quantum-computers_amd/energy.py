"""Energy observable path: the
``autocorr-delta-a-single-qiskit-fast-energy*.py`` family.

The reference builds an L-qubit circuit (no ancilla; optional neel X gates on
qubits 2, 4, ..., L-1 -- ``energy_spec`` / ``engine.energy_init_mask``, even L
raises as the reference does -- then t periods of fast.py's U_F;
energy.py:136-150) and estimates
``<H>`` with ``BackendEstimatorV2`` on AerSimulator under the same
depolarizing model.  ``H`` comes from ``get_hamiltonian`` (energy.py:83-102):

    labels built as strings: position i of "I"*L gets Z (coeff hs[i]),
    positions i, i+1 get ZZ (coeff phis[i]), position i gets X (coeff g*pi).

Qiskit Pauli labels are big-endian — string position i is qubit L-1-i — so
the terms act as ``hs[i] Z_{L-1-i}``, ``phis[i] Z_{L-2-i} Z_{L-1-i}`` and
``g pi X_{L-1-i}``: the fields are applied to the chain in reverse order
relative to the circuit's RZ(hs[i]) on qubit i.  ``hamiltonian_coefficients``
returns the little-endian per-site arrays that reproduce this exactly
(checked against the literal label construction in tests/test_energy_cpu.py).

Execution: one C-ABI call (``dtc_energy``) returns per-trajectory
``<Z_i>(t)``, ``<Z_i Z_i+1>(t)`` and ``<X_i>(t)`` (X basis measured
noiselessly, as Aer executes the estimator's appended basis change outside the
noise model's u1/u2/u3 gates); any Hamiltonian variant of the scripts
("full", "z_only", "zz_only", "x_only", "z_zz") is a linear combination.

Noise accumulation (energy.py:212-218): the script adds
``depolarizing_error(nprob)`` to ONE NoiseModel inside its loop over
``nprobs``, so Aer composes the errors; depolarizing channels compose to
``1 - prod(1 - p_k)``.  ``accumulated_noise`` mirrors that.

Estimator: the reference's ``BackendEstimatorV2`` default precision 1/64
means 4096 shots per measurement basis; here the trajectory mean (each
trajectory an exact expectation) estimates the same quantity.
"""
from __future__ import annotations

import math
import os

import numpy as np

from .engine import SweepSpec, energy_init_mask

HAMILTONIAN_TYPES = ("full", "z_only", "zz_only", "x_only", "z_zz")
ESTIMATOR_SHOTS = int(math.ceil(1.0 / 0.015625 ** 2))  # BackendEstimatorV2 default precision


def hamiltonian_labels(L: int, g: float, hs, phis, hamiltonian_type: str = "full"):
    """The reference's (label, coeff) list, big-endian labels (energy.py:83-102,
    ham-comparison.py:85-115)."""
    if hamiltonian_type not in HAMILTONIAN_TYPES:
        raise ValueError(f"hamiltonian_type must be one of {HAMILTONIAN_TYPES}")
    out = []
    base = "I" * L
    if hamiltonian_type in ("full", "z_only", "z_zz"):
        for i in range(L):
            out.append((base[:i] + "Z" + base[i + 1:], float(hs[i])))
    if hamiltonian_type in ("full", "zz_only", "z_zz"):
        for i in range(L - 1):
            out.append((base[:i] + "ZZ" + base[i + 2:], float(phis[i])))
    if hamiltonian_type in ("full", "x_only"):
        for i in range(L):
            out.append((base[:i] + "X" + base[i + 1:], float(g) * np.pi))
    return out


def hamiltonian_coefficients(L: int, g: float, hs, phis, hamiltonian_type: str = "full"):
    """Little-endian per-site coefficients ``(cz[L], czz[L-1], cx[L])`` with
    ``H = sum_q cz[q] Z_q + sum_q czz[q] Z_q Z_q+1 + sum_q cx[q] X_q``."""
    cz = np.zeros(L)
    czz = np.zeros(max(L - 1, 0))
    cx = np.zeros(L)
    for label, c in hamiltonian_labels(L, g, hs, phis, hamiltonian_type):
        qubits = [L - 1 - i for i, ch in enumerate(label) if ch != "I"]
        kind = label.replace("I", "")
        if kind == "Z":
            cz[qubits[0]] += c
        elif kind == "ZZ":
            czz[min(qubits)] += c
        elif kind == "X":
            cx[qubits[0]] += c
        else:  # pragma: no cover - labels are built above
            raise ValueError(label)
    return cz, czz, cx


def energy_from_observables(obs: dict, L: int, g: float, hs, phis,
                            hamiltonian_type: str = "full") -> np.ndarray:
    """<H> per (..., t) from per-site observables ``z``, ``zz``, ``x``."""
    cz, czz, cx = hamiltonian_coefficients(L, g, hs, phis, hamiltonian_type)
    e = obs["z"] @ cz + obs["x"] @ cx
    if L > 1:
        e = e + obs["zz"] @ czz
    return e


def accumulated_noise(nprobs) -> list:
    """Effective depolarizing parameter of each pass of the reference's loop
    that keeps adding errors to one NoiseModel (energy.py:212-218)."""
    out, keep = [], 1.0
    for p in nprobs:
        keep *= 1.0 - float(p)
        out.append(1.0 - keep)
    return out


def _engine(engine):
    if engine is not None:
        return engine
    from . import sweep

    return sweep._default_engine()


def readout_observables(obs: dict, p01, p10) -> dict:
    """Per-site read-out error on measured expectations: a bit reads 1 for 0
    w.p. p01[i] and 0 for 1 w.p. p10[i], independently, so a measured z_i is
    a_i z_i + b_i in expectation (a = 1 - p01 - p10, b = p10 - p01) and
    z_i z_i+1 -> a_i a_i+1 zz + a_i b_i+1 z_i + b_i a_i+1 z_i+1 + b_i b_i+1.
    X_i is measured after the estimator's basis change: a_i x_i + b_i."""
    p01 = np.asarray(p01, dtype=float)
    p10 = np.asarray(p10, dtype=float)
    a, b = 1.0 - p01 - p10, p10 - p01
    z, zz, x = obs["z"], obs["zz"], obs["x"]
    out = {"z": a * z + b, "x": a * x + b}
    if z.shape[-1] > 1:
        out["zz"] = (a[:-1] * a[1:] * zz + a[:-1] * b[1:] * z[..., :-1]
                     + b[:-1] * a[1:] * z[..., 1:] + b[:-1] * b[1:])
    else:
        out["zz"] = zz
    return out


def energy_spec(L, T, hs, phis, g, initial_state="vacuum", **kw) -> SweepSpec:
    """The energy circuit's sweep: fast.py's periods on L qubits (no ancilla)
    from the energy scripts' own initial state (``energy_init_mask``: neel =
    X on sites 2, 4, ..., L-1, even L raises as in the reference)."""
    return SweepSpec(L=L, T=T, hs=hs, phis=phis, g=g, initial_state=initial_state,
                     init_mask_value=energy_init_mask(L, initial_state), **kw)


def get_instances_energy(spec: SweepSpec, n_traj: int = ESTIMATOR_SHOTS,
                         hamiltonian_types=("full",), seed: int = 0x5EED0001, engine=None,
                         traj_offset: int = 0, readout=None) -> dict:
    """``get_instances`` of the energy scripts: ``<H>(t)`` per instance
    (``[inst][T]``) for each requested Hamiltonian variant, as the trajectory
    mean of the engine's observables (``readout`` = per-site (p01, p10)
    applied to them, device-like noise).  <H> and the read-out map are affine
    in the observables, so the means come from the engine's on-device
    trajectory sums (``energy_sums``, dtc_energy_sums)."""
    sums = _engine(engine).energy_sums(spec, n_traj, seed=seed, traj_offset=traj_offset)
    obs = {k: v / n_traj for k, v in sums.items()}
    if readout is not None:
        obs = readout_observables(obs, *readout)
    out = {}
    for ht in hamiltonian_types:
        out[ht] = np.stack([
            energy_from_observables({k: v[i] for k, v in obs.items()}, spec.L, _g0(spec.g),
                                    spec.hs[i], spec.phis[i], ht)
            for i in range(spec.n_inst)])
    return out


def _g0(g):
    return float(g[0]) if isinstance(g, (list, tuple, np.ndarray)) else float(g)


# ---- the scripts' drivers and output files ---------------------------------------

def energy_folder(L: int, variant: str = "full-ham") -> str:
    """energy.py:59 (``full-ham``), ham-comparison.py:59 (``ham-comparison``),
    energy-fakebrisbane.py:58 (``fakebrisbane``)."""
    return f"energy-data_L{L}-{variant}"


def energy_csv_name(prefix, state, g, L, inst, randomphi, delta, amplitude, noise, use_noise):
    return (f"{prefix}_{state}_g{g}_L{L}_inst{inst}_randomphi{randomphi}_delta{delta}"
            f"_amplitude{amplitude}_noise{noise}_usenoise{use_noise}.csv")


def run_energy(L, g, hs, phis, T, nprobs=(0, 0.001, 0.01, 0.1), use_noise=1,
               initial_state="vacuum", n_traj=ESTIMATOR_SHOTS, seed=0x5EED0001,
               hamiltonian_types=("full",), accumulate=True, engine=None, calibration=None):
    """energy.py's main loop (:212-222): for each nprob, ``av_energy / L`` per
    Hamiltonian variant.  Returns ``{(ht, nprob): [T]}``.

    ``calibration`` (a DeviceCalibration): ``--use_fakebackend 1`` of these
    scripts — ``NoiseModel.from_backend(FakeBrisbane())`` on the simulator,
    where the loop adds no depolarizing error (energy.py:74-78, 214-218): every
    nprob column is the device-noise run (its own shots; here its own seed),
    with per-site read-out error."""
    eff = accumulated_noise(nprobs) if accumulate else [float(p) for p in nprobs]
    res = {}
    for k, (nprob, p_eff) in enumerate(zip(nprobs, eff)):
        spec = energy_spec(L, T, hs, phis, g, initial_state,
                           noise_prob=0.0 if calibration is not None else p_eff,
                           use_noise=1 if calibration is not None else use_noise)
        readout = None
        run_seed = seed
        if calibration is not None:
            spec.device = calibration.device_noise(L)
            readout = calibration.site_readout(L)
            run_seed = seed + 7919 * k
        per = get_instances_energy(spec, n_traj, hamiltonian_types, run_seed, engine,
                                   readout=readout)
        for ht, v in per.items():
            res[(ht, nprob)] = v.mean(axis=0) / L
    return res


def run_energy_device(L, g, hs, phis, T, calibration, initial_state="vacuum",
                      n_traj=ESTIMATOR_SHOTS, seed=0x5EED0001, engine=None):
    """energy-fakebrisbane.py's main loop (:226-234): ``<H>(t)`` under the
    device's noise (here: device-like noise from a calibration file, see
    device_noise.py; FakeBrisbane's own data is unavailable offline), read-out
    error on every measured site, mean over instances — NOT divided by L (the
    script saves ``np.mean(energy, axis=0)`` as is).  ``calibration=None``:
    the script with ``--use_fakebackend 0`` (an empty NoiseModel: noiseless)."""
    spec = energy_spec(L, T, hs, phis, g, initial_state, noise_prob=0.0,
                       use_noise=1 if calibration is not None else 0)
    readout = None
    if calibration is not None:
        spec.device = calibration.device_noise(L)
        readout = calibration.site_readout(L)
    per = get_instances_energy(spec, n_traj if calibration is not None else 1, ("full",), seed,
                               engine, readout=readout)["full"]
    return per.mean(axis=0)


def write_energy_csv(path: str, ts, columns: dict) -> str:
    import pandas as pd

    data = {"time": ts}
    data.update(columns)
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    pd.DataFrame(data).to_csv(path, index=False)
    return path
