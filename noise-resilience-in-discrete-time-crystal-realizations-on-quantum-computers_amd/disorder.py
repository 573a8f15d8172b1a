"""Disorder inputs: ``hs_L{L}.csv`` / ``phis_L{L}.csv`` (consumed unchanged).

* Loading mirrors fast.py:66-74: ``pd.read_csv(comment='#', header=0)``, first
  ``inst`` rows, extra columns ignored by the caller slicing to L / L-1.
* Generation mirrors generate_disorder.py:3-21: ``h ~ U[-pi, pi)``,
  ``phi ~ U[0,1) * A * pi - 1.5 pi + delta * pi`` (or the constant -0.4 when
  ``randomphi != 1``), written with headers ``h_i`` / ``phi_i``
  (generate_disorder.py:24-44).  Unlike the reference, a seed may be given.
"""
from __future__ import annotations

import os

import numpy as np


def load_disorder(L: int, inst: int, folder: str = ".", hs_file: str | None = None,
                  phis_file: str | None = None):
    """Return ``(hs[inst][L], phis[inst][L-1])`` float64 arrays."""
    import pandas as pd

    hs_path = hs_file or os.path.join(folder, f"hs_L{L}.csv")
    phis_path = phis_file or os.path.join(folder, f"phis_L{L}.csv")
    hs_df = pd.read_csv(hs_path, comment="#", header=0)
    phis_df = pd.read_csv(phis_path, comment="#", header=0)
    hs = hs_df.iloc[:inst].values
    phis = phis_df.iloc[:inst].values
    if hs.shape[0] < inst or phis.shape[0] < inst:
        raise ValueError(f"disorder files hold {hs.shape[0]} rows, {inst} instances requested")
    if hs.shape[1] < L or (L > 1 and phis.shape[1] < L - 1):
        raise ValueError(f"disorder files have too few columns for L={L}")
    hs = np.ascontiguousarray(hs[:, :L], dtype=np.float64)
    phis = np.ascontiguousarray(phis[:, : max(L - 1, 0)], dtype=np.float64)
    return hs, phis


def generate_disorder(L: int, inst: int, phi_amplitude: float = 1.0, phi_delta: float = 0.0,
                      randomphi: int = 1, seed: int | None = None):
    rng = np.random.default_rng(seed) if seed is not None else np.random
    hs = rng.random((inst, L)) * 2 * np.pi - np.pi
    if randomphi == 1:
        phis = rng.random((inst, L - 1)) * phi_amplitude * np.pi - 1.5 * np.pi + phi_delta * np.pi
    else:
        phis = np.full((inst, L - 1), -0.4)
    return hs, phis


def save_disorder_to_csv(L: int, inst: int, phi_amplitude: float = 1.0, phi_delta: float = 0.0,
                         randomphi: int = 1, folder: str = ".", seed: int | None = None,
                         hs_name: str | None = None, phis_name: str | None = None):
    import pandas as pd

    hs, phis = generate_disorder(L, inst, phi_amplitude, phi_delta, randomphi, seed)
    os.makedirs(folder, exist_ok=True)
    tag = f"L{L}_inst{inst}_ampl{phi_amplitude}_delta{phi_delta}_randomphi{randomphi}"
    hs_path = os.path.join(folder, hs_name or f"hs_{tag}.csv")
    phis_path = os.path.join(folder, phis_name or f"phis_{tag}.csv")
    pd.DataFrame(hs).to_csv(hs_path, index=False, header=[f"h_{i}" for i in range(hs.shape[1])])
    pd.DataFrame(phis).to_csv(phis_path, index=False,
                              header=[f"phi_{i}" for i in range(phis.shape[1])])
    return hs_path, phis_path
