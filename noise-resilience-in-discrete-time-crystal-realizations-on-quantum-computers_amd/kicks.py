"""Kick-layer specifications: the per-(period, site) gate list of U_F.

Each Floquet period starts with a kick on every site (reference
``create_UF_subcircuit``):

* ``x``  — RX(pi g)                               fast.py:113-114
* ``y``  — RY(pi g)                               ...-polarization.py:115-116
* ``xy`` — RX(pi g/2) then RY(pi g/2)             ...-polarization.py:117-119
* ``yx`` — RY(pi g/2) then RX(pi g/2)             ...-polarization.py:120-122
* ``circular_left/right`` — RX(pi g cos(w s)/sqrt2) then RY(+-pi g sin(w s)/sqrt2),
  s = period index from 0                          ...-circular-polarization.py:123-136
* ``circular_static`` — RX(pi g/sqrt2) then RY(pi g/sqrt2)  ...:137-141
* ``xy_cycle`` — x for periods s//5 even, y for odd  ...-polarization-xy-cycle.py:144-147
* per-period ``g`` list (controlled-g)             ...-controlled-g.py:215-227

Every sub-gate transpiles to one noisy ``u3``, so each sub-gate
is followed by a depolarizing draw in the engine.  The table layout is
``[n_periods][L][n_sub][8]`` float64 (complex 2x2, row-major, interleaved),
row ``s`` = the ``(s+1)``-th forward period.
"""
from __future__ import annotations

import math
from typing import Sequence

import numpy as np

POLARIZATIONS = ("x", "y", "xy", "yx", "circular_left", "circular_right", "circular_static",
                 "xy_cycle")


def rx(theta: float) -> np.ndarray:
    """qiskit RXGate(theta) = [[c, -i s], [-i s, c]]."""
    c, s = math.cos(theta / 2), math.sin(theta / 2)
    return np.array([[c, -1j * s], [-1j * s, c]], dtype=np.complex128)


def ry(theta: float) -> np.ndarray:
    """qiskit RYGate(theta) = [[c, -s], [s, c]]."""
    c, s = math.cos(theta / 2), math.sin(theta / 2)
    return np.array([[c, -s], [s, c]], dtype=np.complex128)


def period_gate_specs(polarization: str, g: float, step: int, circular_frequency: float = 1.0):
    """Sub-gate list [(name, angle)] (application order) of one site's kick at
    period index ``step`` (0-based)."""
    pg = math.pi * g
    if polarization == "x":
        return [("rx", pg)]
    if polarization == "y":
        return [("ry", pg)]
    if polarization == "xy":
        return [("rx", pg / 2), ("ry", pg / 2)]
    if polarization == "yx":
        return [("ry", pg / 2), ("rx", pg / 2)]
    if polarization in ("circular_left", "circular_right"):
        w = circular_frequency
        ax = pg * math.cos(w * step) / math.sqrt(2)
        ay = pg * math.sin(w * step) / math.sqrt(2)
        if polarization == "circular_right":
            ay = -ay
        return [("rx", ax), ("ry", ay)]
    if polarization == "circular_static":
        return [("rx", pg / math.sqrt(2)), ("ry", pg / math.sqrt(2))]
    if polarization == "xy_cycle":
        return [("rx", pg)] if (step // 5) % 2 == 0 else [("ry", pg)]
    raise ValueError(f"unknown polarization {polarization!r}; expected one of {POLARIZATIONS}")


def period_gates(polarization: str, g: float, step: int, circular_frequency: float = 1.0):
    """Sub-gate matrices (application order) of one site's kick at period ``step``."""
    return [rx(a) if n == "rx" else ry(a)
            for n, a in period_gate_specs(polarization, g, step, circular_frequency)]


def kick_table(L: int, n_periods: int, g: float | Sequence[float] = 0.97,
               polarization: str = "x", circular_frequency: float = 1.0) -> np.ndarray:
    """Build the ``[n_periods][L][n_sub][8]`` kick table.

    ``g`` may be a scalar or a per-period list (``g[s]`` used at period index s,
    controlled-g.py:215-227; shorter lists fall back to ``g[0]`` as there).
    """
    n_periods = max(1, int(n_periods))
    rows = []
    for s in range(n_periods):
        if isinstance(g, (list, tuple, np.ndarray)):
            gs = float(g[s]) if len(g) > s else (float(g[0]) if len(g) else 0.84)
        else:
            gs = float(g)
        rows.append(period_gates(polarization, gs, s, circular_frequency))
    n_sub = max(len(r) for r in rows)
    tab = np.zeros((n_periods, L, n_sub, 8), dtype=np.float64)
    for s, gates in enumerate(rows):
        # every sub-gate carries its own noise draw, so the count must not vary
        if len(gates) != n_sub:
            raise ValueError("kick sub-gate count must be constant over periods")
        for q, m in enumerate(gates):
            tab[s, :, q, :] = matrix_to_row(m)
    return np.ascontiguousarray(tab)


def matrix_to_row(m: np.ndarray) -> np.ndarray:
    """complex 2x2 -> interleaved float64[8] (ABI layout)."""
    m = np.asarray(m, dtype=np.complex128).reshape(4)
    return np.stack([m.real, m.imag], axis=-1).reshape(8)


def row_to_matrix(r: np.ndarray) -> np.ndarray:
    r = np.asarray(r, dtype=np.float64).reshape(4, 2)
    return (r[:, 0] + 1j * r[:, 1]).reshape(2, 2)


def n_sub_of(polarization: str) -> int:
    return len(period_gates(polarization, 1.0, 0))
