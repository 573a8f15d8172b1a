"""Device-like noise: the build's stand-in for ``use_fakebackend=1``.

The reference's ``--use_fakebackend 1`` (fast.py:77-79, 152-153) builds
``NoiseModel.from_backend(FakeBrisbane())``: per-qubit thermal relaxation
(T1, T2, gate length) plus depolarizing gate errors and read-out errors from
an IBM calibration snapshot that ships inside ``qiskit_ibm_runtime`` — not
installed here and not fetchable offline.  The build takes
the same physics from a calibration file the user supplies (JSON, schema
below; ``data/device_standin_L20.json`` is a documented stand-in with
Eagle-class values, NOT Brisbane's data) and runs it through the
``dtc_autocorr_device`` C ABI (include/dtc.h):

* after every kick sub-gate on site i: amplitude damping
  gamma_i = 1 - exp(-t_kick / T1_i), pure dephasing to the total coherence
  decay exp(-t_kick / T2_i), then depolarizing_error(p_i, 1);
* the ancilla (Hadamard-test qubit) enters through ``anc_factor`` (its six
  single-qubit gates and two CZs, each a depolarizing channel that scales the
  measured coherence) and its read-out assignment errors.

Parity with the reference is unpinned: no FakeBrisbane output exists in the
reference tree (the draw script's autocorr_data_L20_fakebrisbane/ is absent)
and the routed ECR circuit of a real backend differs from the folded model.
What the tests pin is the model itself: engine vs the C oracle per
trajectory, and trajectory means vs the exact density matrix.

Calibration JSON schema::

    {"name": str, "note": str,
     "sx_gate_ns": float,            # duration of one sx pulse
     "kick_sx_count": int,           # sx pulses per RX/RY kick (rz-sx-rz-sx-rz: 2)
     "qubits": [                     # circuit order: [0] = ancilla, [1 + i] = site i
        {"T1_us": float, "T2_us": float, "sx_error": float,
         "readout_p01": float, "readout_p10": float}, ...],
     "cz_error": float}              # two-qubit (ancilla-site) gate error
"""
from __future__ import annotations

import json
from dataclasses import dataclass

import numpy as np


@dataclass
class DeviceNoise:
    """Per-site channel parameters for ``dtc_autocorr_device`` (include/dtc.h)."""

    p_gate: np.ndarray       # [L] depolarizing parameter per kick sub-gate
    t1_us: np.ndarray        # [L]
    t2_us: np.ndarray        # [L]
    gate_ns: float           # duration of one kick sub-gate
    anc_factor: float = 1.0  # ancilla coherence factor
    readout_p01: float = 0.0
    readout_p10: float = 0.0

    def __post_init__(self):
        self.p_gate = np.ascontiguousarray(self.p_gate, dtype=np.float64)
        self.t1_us = np.ascontiguousarray(self.t1_us, dtype=np.float64)
        self.t2_us = np.ascontiguousarray(self.t2_us, dtype=np.float64)
        if not (self.p_gate.shape == self.t1_us.shape == self.t2_us.shape):
            raise ValueError("p_gate, t1_us, t2_us must have one entry per site")

    @property
    def L(self) -> int:
        return int(self.p_gate.shape[0])

    def site_channels(self):
        """Per-site (gamma, dephasing Z probability, depolarizing p): the same
        formulas as the engine (dtc_engine.cpp setup_device_noise)."""
        out = []
        for p, t1u, t2u in zip(self.p_gate, self.t1_us, self.t2_us):
            t1 = t1u * 1e3 if t1u > 0 else np.inf
            t2 = t2u * 1e3 if t2u > 0 else np.inf
            t2 = min(t2, 2.0 * t1)
            tg = self.gate_ns
            gamma = 0.0 if np.isinf(t1) else 1.0 - np.exp(-tg / t1)
            rate = (0.0 if np.isinf(t2) else 1.0 / t2) - (0.0 if np.isinf(t1) else 0.5 / t1)
            d = 0.5 * (1.0 - np.exp(-tg * max(0.0, rate)))
            out.append((float(gamma), float(d), float(p)))
        return out

    def readout(self, a):
        """Ancilla read-out of expectation(s) a: (1 - p01 - p10) a + (p10 - p01)."""
        return (1.0 - self.readout_p01 - self.readout_p10) * np.asarray(a) + (
            self.readout_p10 - self.readout_p01)


def depolarizing_param(error: float, n_qubits: int = 1) -> float:
    """Aer depolarizing parameter with average gate infidelity ``error``:
    F_avg = 1 - p (d - 1) / d, so 1 qubit p = 2 e, 2 qubits p = 4 e / 3."""
    d = 2 ** n_qubits
    return error * d / (d - 1)


@dataclass
class DeviceCalibration:
    """A calibration file (schema in the module docstring)."""

    name: str
    qubits: list
    sx_gate_ns: float
    kick_sx_count: int = 2
    cz_error: float = 0.0
    note: str = ""

    @classmethod
    def from_json(cls, path: str) -> "DeviceCalibration":
        with open(path) as f:
            d = json.load(f)
        return cls(name=d.get("name", "device"), qubits=list(d["qubits"]),
                   sx_gate_ns=float(d["sx_gate_ns"]), kick_sx_count=int(d.get("kick_sx_count", 2)),
                   cz_error=float(d.get("cz_error", 0.0)), note=d.get("note", ""))

    def site_readout(self, L: int):
        """Per-site read-out flip probabilities (p01[L], p10[L]) of the chain
        qubits (qubits[1..L]): the energy estimator measures every site."""
        if len(self.qubits) < L + 1:
            raise ValueError(f"calibration {self.name!r} has {len(self.qubits)} qubits, "
                             f"need {L + 1} (ancilla + {L} sites)")
        sites = self.qubits[1:L + 1]
        return (np.array([float(q.get("readout_p01", 0.0)) for q in sites]),
                np.array([float(q.get("readout_p10", 0.0)) for q in sites]))

    def device_noise(self, L: int, n_anc_1q: int = 6, n_anc_2q: int = 2) -> DeviceNoise:
        """Channel parameters for an L-site chain (qubits[1..L]) with the
        ancilla on qubits[0].  A kick = ``kick_sx_count`` sx pulses: error
        and duration scale with it.  Ancilla factor = (1 - p1)^n_anc_1q
        (1 - p2)^n_anc_2q: every depolarizing channel scales the measured
        coherence by (1 - p) (fast.py's (1 - p)^6 is the n_anc_2q = 0 case)."""
        if len(self.qubits) < L + 1:
            raise ValueError(f"calibration {self.name!r} has {len(self.qubits)} qubits, "
                             f"need {L + 1} (ancilla + {L} sites)")
        sites = self.qubits[1:L + 1]
        n = self.kick_sx_count
        p_gate = [depolarizing_param(min(0.75, n * q["sx_error"])) for q in sites]
        anc = self.qubits[0]
        p1 = depolarizing_param(anc["sx_error"])
        p2 = depolarizing_param(self.cz_error, 2)
        return DeviceNoise(
            p_gate=np.array(p_gate), t1_us=np.array([q["T1_us"] for q in sites]),
            t2_us=np.array([q["T2_us"] for q in sites]), gate_ns=n * self.sx_gate_ns,
            anc_factor=(1.0 - p1) ** n_anc_1q * (1.0 - p2) ** n_anc_2q,
            readout_p01=float(anc.get("readout_p01", 0.0)),
            readout_p10=float(anc.get("readout_p10", 0.0)))
