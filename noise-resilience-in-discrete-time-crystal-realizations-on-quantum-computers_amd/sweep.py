"""Sweep drivers and on-disk artefacts of autocorr-delta-a-single-qiskit-fast.py.

* ``get_single_out`` / ``get_instances`` mirror fast.py:217-239 (same names,
  same return shapes ``[T]`` / ``[inst][T]``), but one engine call produces
  every t of every instance.
* ``compute_z_expectation`` mirrors fast.py:92-109.
* ``autocorr_csv_path`` / ``write_autocorr_csv`` reproduce the folder, file
  name and columns of fast.py:56-59, 259-270 so draw-*.py read our output
  unchanged.
* ``write_gate_counts`` reproduces gate_counts_*.csv (fast.py:193-197).

Estimators: with ``shots=None`` the value per (instance, t) is the
trajectory mean of the ancilla expectation (lower variance than the
reference).  With ``shots=S`` each of S trajectories contributes one
simulated ancilla measurement, i.e. the exact distribution of the
reference's ``(n0 - n1)/S`` (fast.py:211-213); noiseless runs use one exact
statevector and a Binomial(S, (1+A)/2) draw, as Aer does for ideal circuits.
"""
from __future__ import annotations

import os
import dataclasses
from dataclasses import dataclass

import numpy as np

from .circuit import dtc_circuit, transpile_aer_basis
from .engine import DtcEngine, SweepSpec
from .kicks import period_gate_specs


def compute_z_expectation(counts: dict, num_qubits: int):
    """fast.py:92-109: per-qubit (p0 - p1)/shots, qiskit little-endian keys."""
    total_shots = sum(counts.values())
    out = []
    for qubit in range(num_qubits):
        p0 = p1 = 0
        for bitstring, count in counts.items():
            if bitstring[::-1][qubit] == "0":
                p0 += count
            else:
                p1 += count
        out.append((p0 - p1) / total_shots)
    return out


@dataclass
class SweepResult:
    fwd: np.ndarray | None        # [n_inst][T] per-instance estimates
    echo: np.ndarray | None       # [n_inst][T]
    fwd_traj: np.ndarray | None   # [n_inst][n_traj][T] per-trajectory values
    echo_traj: np.ndarray | None
    zsite: np.ndarray | None      # [n_inst][n_traj][T][L]

    @property
    def av_autocorr(self):
        return None if self.fwd is None else np.mean(self.fwd, axis=0)

    @property
    def av_autocorr_echo(self):
        return None if self.echo is None else np.mean(self.echo, axis=0)


def _shot_estimate(a: np.ndarray, shots: int, rng: np.random.Generator) -> np.ndarray:
    """a: [n_inst][n_traj][T] per-trajectory ancilla expectations -> [n_inst][T]."""
    n_inst, n_traj, T = a.shape
    if n_traj == 1:
        n0 = rng.binomial(shots, np.clip((1.0 + a[:, 0, :]) / 2.0, 0.0, 1.0))
        return (2.0 * n0 - shots) / shots
    if n_traj != shots:
        raise ValueError("shot emulation needs n_traj == shots (one trajectory per shot)")
    u = rng.random(a.shape)
    zero = u < (1.0 + a) / 2.0
    return (2.0 * zero.sum(axis=1) - shots) / shots


def point_seed(seed: int, t: int) -> int:
    """The Philox key of time point t in the independent-per-t mode: a
    splitmix64 finaliser of (seed, t), so every point draws from its own key
    whatever trajectory ids a caller's chunks use."""
    m = (1 << 64) - 1
    z = (seed + (t + 1) * 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    return z ^ (z >> 31)


def autocorr_independent_t(eng, spec: SweepSpec, n_traj: int, seed: int = 0x5EED0001,
                           lo: int = 0, want_fwd=True, want_echo=True, batch: int = 0) -> dict:
    """Per-trajectory outputs like ``eng.autocorr``, but every time point from
    its own trajectories, as the reference's fresh circuit per t
    (autocorr-delta-a-single-qiskit-fast.py:219-221): point t runs a sweep of
    t + t_offset periods that measures only t (``t_first``) under its own key
    ``point_seed(seed, t)``, trajectory ids lo .. lo + n_traj - 1 -- so the
    points share no noise draw across t, and chunks of one run split by
    trajectory offset (``lo``) compose to the single-call values.  Costs O(T^2)
    period applications instead of O(T^2 / 2) shared with the forward branch:
    about 2 t periods per trajectory for point t."""
    n_inst, T = spec.n_inst, spec.T
    out = {}
    if want_fwd:
        out["fwd"] = np.zeros((n_inst, n_traj, T))
    if want_echo:
        out["echo"] = np.zeros((n_inst, n_traj, T))
    for t in range(T):
        rows = max(1, t + spec.t_offset)
        s_t = dataclasses.replace(spec, T=t + 1, kick=spec.kick[:rows])
        r = eng.autocorr(s_t, n_traj, seed=point_seed(seed, t), traj_offset=lo,
                         want_fwd=want_fwd, want_echo=want_echo, batch=batch, t_first=t)
        for k in out:
            out[k][:, :, t] = r[k][:, :, t]
    return out


def run_sweep(spec: SweepSpec, n_traj: int | None = None, shots: int | None = None,
              engine: DtcEngine | None = None, seed: int = 0x5EED0001, want_fwd=True,
              want_echo=True, want_zsite=False, traj_offset: int = 0,
              batch: int = 0, independent_t: bool = False) -> SweepResult:
    """All t of all instances in one engine call (``independent_t``: one call
    per t with its own trajectories, ``autocorr_independent_t``)."""
    eng = engine or _default_engine()
    if n_traj is None:
        n_traj = 1 if (spec.p == 0 and spec.device is None) else (shots or 1024)
    if independent_t:
        if want_zsite:
            raise ValueError("independent_t: per-site Z is a forward-sweep output")
        out = autocorr_independent_t(eng, spec, n_traj, seed=seed, lo=traj_offset,
                                     want_fwd=want_fwd, want_echo=want_echo, batch=batch)
    else:
        out = eng.autocorr(spec, n_traj, seed=seed, traj_offset=traj_offset, want_fwd=want_fwd,
                           want_echo=want_echo, want_zsite=want_zsite, batch=batch)
    rng = np.random.default_rng(seed)
    res = {}
    for key in ("fwd", "echo"):
        if key not in out:
            res[key] = None
            continue
        a = out[key]
        if shots is None:
            res[key] = a.mean(axis=1)
        elif spec.device is not None:
            # device-like noise: importance-weighted trajectories are not
            # per-shot probabilities; draw the shots from the trajectory mean
            m = np.clip((1.0 + a.mean(axis=1)) / 2.0, 0.0, 1.0)
            res[key] = (2.0 * rng.binomial(shots, m) - shots) / shots
        else:
            res[key] = _shot_estimate(a, shots, rng)
    return SweepResult(res["fwd"], res["echo"], out.get("fwd"), out.get("echo"),
                       out.get("zsite"))


_ENGINE = None


def _default_engine():
    global _ENGINE
    if _ENGINE is None:
        _ENGINE = DtcEngine(int(os.environ.get("LOCAL_RANK", "0")))
    return _ENGINE


def get_instances(spec: SweepSpec, echo: bool, shots: int | None = 1024, **kw):
    """fast.py:228-239 — returns [inst][T]."""
    r = run_sweep(spec, shots=shots, want_fwd=not echo, want_echo=echo, **kw)
    return r.echo if echo else r.fwd


def get_single_out(spec: SweepSpec, inst_number: int, echo: bool, shots: int | None = 1024,
                   **kw):
    """fast.py:217-224 — returns [T] for one instance."""
    # every field carries over (device-like noise, polarization, ...)
    one = dataclasses.replace(spec, hs=spec.hs[inst_number:inst_number + 1],
                              phis=spec.phis[inst_number:inst_number + 1])
    return get_instances(one, echo, shots=shots, **kw)[0]


# -- artefacts -------------------------------------------------------------
def folder_name(L, noise_prob, use_fakebackend=0):
    """fast.py:56."""
    return f"autocorr_data_L{L}_noiseprob{noise_prob}_fakebackend{use_fakebackend}"


def autocorr_csv_name(state, g, L, inst, tf, randomphi, phi_delta, phi_amplitude, noise_prob,
                      use_noise):
    """fast.py:266."""
    return (f"autocorr_data_{state}_g{g}_L{L}_inst{inst}_tf{tf}_randomphi{randomphi}"
            f"_delta{phi_delta}_amplitude{phi_amplitude}_noise{noise_prob}_usenoise{use_noise}.csv")


def write_autocorr_csv(path, ts, av_autocorr, av_autocorr_echo):
    """fast.py:259-269: columns time, av_autocorr, av_autocorr_echo,
    sqrt_av_autocorr_echo; index=False; sqrt of negatives -> NaN (empty)."""
    import pandas as pd

    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with np.errstate(invalid="ignore"):
        sq = np.sqrt(av_autocorr_echo)
    df = pd.DataFrame({
        "time": ts,
        "av_autocorr": av_autocorr,
        "av_autocorr_echo": av_autocorr_echo,
        "sqrt_av_autocorr_echo": sq,
    })
    df.to_csv(path, index=False)
    return path


def gate_counts_name(t, echo, backend_name="aer_simulator", tag="iqm"):
    """fast.py:196 (routing None is printed via routing_method='lookahead')."""
    echo_str = "echo" if echo else "forward"
    return (f"gate_counts_t{t}_{echo_str}_opt0_{backend_name}_coupling_routelookahead_"
            f"layoutdense_{tag}.csv")


def write_gate_counts(folder, spec: SweepSpec, polarization="x", g=0.97, tag="iqm",
                      circular_frequency=1.0):
    """Write gate_counts_t{t}_{forward,echo}_*.csv for t < T exactly as the
    reference's transpile + count_ops does (fast.py:192-197)."""
    import pandas as pd

    os.makedirs(folder, exist_ok=True)
    paths = []

    def kick_layers(step):
        return period_gate_specs(polarization, g, step, circular_frequency)

    for echo in (False, True):
        for t in range(spec.T):
            circ = dtc_circuit(spec.L, t + spec.t_offset, spec.hs[0], spec.phis[0], kick_layers,
                               echo=echo, initial_state=spec.initial_state,
                               probe=spec.probe_site)
            counts = transpile_aer_basis(circ).count_ops()
            p = os.path.join(folder, gate_counts_name(t, echo, tag=tag))
            pd.DataFrame(list(counts.items()), columns=["gate", "count"]).to_csv(p, index=False)
            paths.append(p)
    return paths
