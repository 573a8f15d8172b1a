"""Minimal circuit IR mirroring the subset of ``qiskit.QuantumCircuit`` the
reference's DTC scripts use, and the gate-count semantics of their
transpilation.

Reference usage (autocorr-delta-a-single-qiskit-fast.py):
  QuantumCircuit(L+1, 1)                                   :125
  .x / .h / .cz / .rx / .ry / .rzz / .rz / .measure        :113-147
  .append(UF_subcircuit, range(L+1)), UF.inverse()         :135-143
  generate_preset_pass_manager(optimization_level=0, backend=AerSimulator(...),
     routing_method=None, initial_layout=...) .run(circ)   :181-192
  circ_tnoise.count_ops() -> gate_counts_*.csv             :193-197

The transpiler is restated only as far as its OUTPUT is observable on this
path: Aer restricts the basis to the noise-model gates, so (pinned by all
182 ``gate_counts_*aer_simulator*.csv`` files of the reference)
  rx, ry, x -> u3;  h -> u2;  cz -> u2 . cx . u2 (u2 on the target);
  rzz -> cx . rz . cx;  rz -> rz;  measure -> measure.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Iterable, Sequence

_SELF_INVERSE = {"x", "h", "cz", "cx", "y", "z"}
_ROTATIONS = {"rx", "ry", "rz", "rzz"}


@dataclass(frozen=True)
class Instruction:
    name: str
    qubits: tuple
    params: tuple = ()
    clbits: tuple = ()

    @property
    def operation(self):  # qiskit CircuitInstruction-like access
        return self


class QuantumCircuit:
    """Gate list over ``num_qubits`` qubits (qubit q = bit q, little-endian)."""

    def __init__(self, num_qubits: int, num_clbits: int = 0, name: str | None = None):
        self.num_qubits = int(num_qubits)
        self.num_clbits = int(num_clbits)
        self.name = name or "circuit"
        self.data: list[Instruction] = []

    # -- qiskit-like accessors ----------------------------------------
    @property
    def qubits(self):
        return list(range(self.num_qubits))

    def __len__(self):
        return len(self.data)

    def _q(self, q):
        q = int(q)
        if not 0 <= q < self.num_qubits:
            raise IndexError(f"qubit {q} out of range for {self.num_qubits}-qubit circuit")
        return q

    def _add(self, name, qubits, params=(), clbits=()):
        self.data.append(Instruction(name, tuple(self._q(q) for q in qubits),
                                     tuple(float(p) for p in params), tuple(clbits)))
        return self

    # -- gates used by the reference ------------------------------------
    def x(self, q):
        return self._add("x", (q,))

    def h(self, q):
        return self._add("h", (q,))

    def cz(self, a, b):
        return self._add("cz", (a, b))

    def cx(self, a, b):
        return self._add("cx", (a, b))

    def rx(self, theta, q):
        return self._add("rx", (q,), (theta,))

    def ry(self, theta, q):
        return self._add("ry", (q,), (theta,))

    def rz(self, theta, q):
        return self._add("rz", (q,), (theta,))

    def rzz(self, theta, a, b):
        return self._add("rzz", (a, b), (theta,))

    def measure(self, q, c):
        if not 0 <= int(c) < self.num_clbits:
            raise IndexError("classical bit out of range")
        return self._add("measure", (q,), (), (int(c),))

    def barrier(self, *qargs):
        return self

    # -- composition ------------------------------------------------------
    def append(self, other: "QuantumCircuit", qargs: Iterable[int], cargs=None):
        qargs = list(qargs)
        if not isinstance(other, QuantumCircuit):
            raise TypeError("append expects a QuantumCircuit (sub-circuit)")
        if len(qargs) != other.num_qubits:
            raise ValueError("qargs length must equal the appended circuit's width")
        for ins in other.data:
            if ins.name == "measure":
                raise ValueError("cannot append a sub-circuit with measurements")
            self._add(ins.name, [qargs[q] for q in ins.qubits], ins.params)
        return self

    compose = append

    def inverse(self) -> "QuantumCircuit":
        inv = QuantumCircuit(self.num_qubits, self.num_clbits, self.name + "_dg")
        for ins in reversed(self.data):
            if ins.name == "measure":
                raise ValueError("cannot invert a circuit with measurements")
            if ins.name in _SELF_INVERSE:
                inv._add(ins.name, ins.qubits)
            elif ins.name in _ROTATIONS:
                inv._add(ins.name, ins.qubits, tuple(-p for p in ins.params))
            else:
                raise ValueError(f"cannot invert gate {ins.name}")
        return inv

    def copy(self):
        c = QuantumCircuit(self.num_qubits, self.num_clbits, self.name)
        c.data = list(self.data)
        return c

    def count_ops(self) -> "OrderedDict[str, int]":
        """qiskit semantics: counts sorted by count, descending (stable)."""
        counts: dict[str, int] = {}
        for ins in self.data:
            counts[ins.name] = counts.get(ins.name, 0) + 1
        return OrderedDict(sorted(counts.items(), key=lambda kv: kv[1], reverse=True))


# -- transpilation to the Aer noise basis ------------------------------------
_BASIS_MAP = {
    "rx": ("u3",),
    "ry": ("u3",),
    "x": ("u3",),
    "h": ("u2",),
    "cz": ("u2", "cx", "u2"),
    "rzz": ("cx", "rz", "cx"),
    "rz": ("rz",),
    "cx": ("cx",),
    "measure": ("measure",),
}


def transpile_aer_basis(circ: QuantumCircuit) -> QuantumCircuit:
    """Gate-level output of the reference's preset pass manager at
    optimization_level=0 for the Aer backend restricted to the u1/u2/u3
    noise basis (fast.py:181-192): same gate multiset and first-appearance
    order as qiskit produces for these circuits.  Parameters of the basis
    gates are not needed by anything on this path and are dropped."""
    out = QuantumCircuit(circ.num_qubits, circ.num_clbits, circ.name)
    for ins in circ.data:
        names = _BASIS_MAP.get(ins.name)
        if names is None:
            raise ValueError(f"gate {ins.name} not in the DTC gate set")
        for nm in names:
            if nm == "measure":
                out.data.append(Instruction("measure", ins.qubits, (), ins.clbits))
            elif nm == "cx":
                q = ins.qubits if len(ins.qubits) == 2 else (ins.qubits[0], ins.qubits[0])
                out.data.append(Instruction("cx", q))
            elif nm in ("u2",) and ins.name == "cz":
                out.data.append(Instruction("u2", (ins.qubits[1],)))
            elif nm == "rz" and ins.name == "rzz":
                out.data.append(Instruction("rz", (ins.qubits[1],), ins.params))
            else:
                out.data.append(Instruction(nm, (ins.qubits[0],), ins.params))
    return out


def gate_counts_closed_form(L: int, periods: int, kick_gates_per_site: int = 1,
                            neel: bool = False) -> "OrderedDict[str, int]":
    """Closed form of the transpiled counts:
    cx = 2 + 2(L-1)P, rz = (2L-1)P, u3 = k L P (+ L/2 neel X), u2 = 6, measure = 1."""
    P = periods
    d = {"u2": 6, "cx": 2 + 2 * (L - 1) * P, "rz": (2 * L - 1) * P,
         "u3": kick_gates_per_site * L * P + (L // 2 if neel else 0), "measure": 1}
    d = {k: v for k, v in d.items() if v}
    return OrderedDict(sorted(d.items(), key=lambda kv: kv[1], reverse=True))


def dtc_circuit(L: int, t: int, hs: Sequence[float], phis: Sequence[float],
                kick_layers, echo: bool = False, initial_state: str = "vacuum",
                probe: int | None = None) -> QuantumCircuit:
    """Build the reference's ancilla autocorrelator circuit (fast.py:124-147)
    with this IR.  ``kick_layers(step)`` returns the per-site list of
    (gate_name, angle) sub-gates of period index ``step``."""
    j = int(L / 2) if probe is None else probe
    circ = QuantumCircuit(L + 1, 1)
    if initial_state == "neel":
        for i in range(1, L + 1):
            if i % 2 == 0:
                circ.x(i)
    circ.h(0)
    circ.cz(j + 1, 0)

    def uf(step):
        sub = QuantumCircuit(L + 1)
        gates = kick_layers(step)
        for i in range(L):
            for name, ang in gates:
                getattr(sub, name)(ang, i + 1)
        for i in range(0, L - 1, 2):
            sub.rzz(phis[i], i + 1, i + 2)
        for i in range(1, L - 1, 2):
            sub.rzz(phis[i], i + 1, i + 2)
        for i in range(L):
            sub.rz(hs[i], i + 1)
        return sub

    for step in range(t):
        circ.append(uf(step), range(L + 1))
    if echo:
        for step in range(t - 1, -1, -1):
            circ.append(uf(step).inverse(), range(L + 1))
    circ.cz(j + 1, 0)
    circ.h(0)
    circ.measure(0, 0)
    return circ
