"""AerSimulator-shaped drop-in facade over the HIP engine.

The reference's call sites (autocorr-delta-a-single-qiskit-fast.py):
    noise_model = NoiseModel()                                         :76
    error = depolarizing_error(noise_prob, 1)                          :85
    noise_model.add_all_qubit_quantum_error(error, ["u1","u2","u3"])   :86
    backend = AerSimulator(noise_model=noise_model, device="GPU",
                           cuStateVec_enable=True)                     :156
    result = backend.run(circ_tnoise, shots=1024).result()             :211
    counts = result.get_counts(circ_tnoise)                            :212
work unchanged against ``DtcSimulator`` (alias ``AerSimulator``) and the
``NoiseModel`` / ``depolarizing_error`` classes here, with circuits built by
``circuit.QuantumCircuit``.  ``run`` folds the (L+1)-qubit Hadamard-test
circuit onto the L-qubit engine: each shot is one noisy
trajectory of the system plus one Bernoulli draw of the ancilla outcome with
P(0) = (1 + a_r)/2, a_r = (1-p)^6 z_j <Z_j>_r, which is exactly the
distribution of Aer's shots.  Circuits outside that family raise
``NotImplementedError`` (no silent fallback).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from .circuit import QuantumCircuit
from .engine import DtcEngine, SweepSpec
from .kicks import matrix_to_row, rx as rx_m, ry as ry_m

_KICK_GATES = {"rx", "ry"}
_DIAG_GATES = {"rz", "rzz"}
# gate -> Aer basis gate that carries its noise (fast.py:84-86 + transpile)
_NOISE_CARRIER = {"rx": "u3", "ry": "u3", "x": "u3", "h": "u2"}


class QuantumError:
    def __init__(self, kind: str, p: float, num_qubits: int):
        self.kind, self.p, self.num_qubits = kind, float(p), int(num_qubits)

    def __repr__(self):
        return f"QuantumError({self.kind}, p={self.p}, n={self.num_qubits})"


def depolarizing_error(param: float, num_qubits: int) -> QuantumError:
    """qiskit_aer.noise.depolarizing_error: rho -> (1-p) rho + p I/2^n."""
    if num_qubits != 1:
        raise NotImplementedError("only single-qubit depolarizing errors occur on this path")
    if not 0.0 <= param <= 4.0 / 3.0:
        raise ValueError("depolarizing parameter must be in [0, 4/3]")
    return QuantumError("depolarizing", param, num_qubits)


class NoiseModel:
    """Subset of qiskit_aer.noise.NoiseModel used by the reference."""

    def __init__(self, basis_gates=None):
        self._errors: dict[str, QuantumError] = {}
        self.basis_gates = list(basis_gates or ["id", "rz", "sx", "cx"])

    def add_all_qubit_quantum_error(self, error: QuantumError, instructions, warnings=True):
        if isinstance(instructions, str):
            instructions = [instructions]
        for g in instructions:
            self._errors[g] = error

    @classmethod
    def from_backend(cls, backend, **kw):
        """fast.py:77-79.  FakeBrisbane's calibration ships inside
        qiskit_ibm_runtime (not available offline); a ``FakeDevice`` built
        from a calibration file gives the device-like noise path instead."""
        if not isinstance(backend, FakeDevice):
            raise NotImplementedError(
                "NoiseModel.from_backend needs calibration data: FakeBrisbane's is not "
                "available offline; use FakeDevice(<calibration.json>) "
                "(data/device_standin_L20.json is a documented stand-in)")
        nm = cls(basis_gates=["ecr", "id", "rz", "sx", "x"])
        nm.device_calibration = backend.calibration
        return nm

    device_calibration = None

    @property
    def noise_instructions(self):
        return sorted(self._errors)

    def error_for(self, gate: str):
        carrier = _NOISE_CARRIER.get(gate)
        return self._errors.get(carrier) if carrier else None

    def is_ideal(self):
        return not self._errors and self.device_calibration is None


class FakeDevice:
    """A backend-like calibration holder for NoiseModel.from_backend (the
    stand-in for fast.py's FakeBrisbane(), device_noise.py)."""

    def __init__(self, calibration_path: str):
        from .device_noise import DeviceCalibration

        self.calibration = DeviceCalibration.from_json(calibration_path)
        self.name = self.calibration.name
        self.num_qubits = len(self.calibration.qubits)


@dataclass
class FoldedCircuit:
    """An ancilla autocorrelator circuit mapped to the engine's inputs."""

    L: int
    n_fwd: int
    echo: bool
    probe: int
    init_mask: int
    hs: np.ndarray
    phis: np.ndarray
    kick: np.ndarray        # [max(1,n_fwd)][L][n_sub][8]
    kick_noisy: bool
    n_anc_noisy: int
    prep_noisy: bool


def _site_of(q: int, anc: int) -> int:
    return q - 1 if q > anc else q


def fold_circuit(circ: QuantumCircuit, noise: NoiseModel | None) -> FoldedCircuit:
    """Recognise fast.py:124-147's circuit family (any kick polarization, any
    per-period kick list, optional echo, vacuum/neel prep) and extract the
    engine problem.  Raises NotImplementedError for anything else."""
    noise = noise or NoiseModel()
    data = list(circ.data)
    meas = [k for k, ins in enumerate(data) if ins.name == "measure"]
    if len(meas) != 1 or meas[0] != len(data) - 1:
        raise NotImplementedError("expected exactly one final measurement (of the ancilla)")
    anc = data[-1].qubits[0]
    n = circ.num_qubits
    L = n - 1
    k = 0
    init = 0
    prep_noisy = False
    while k < len(data) and data[k].name == "x":
        q = data[k].qubits[0]
        if q == anc:
            raise NotImplementedError("X on the ancilla is not part of the DTC protocol")
        init |= 1 << _site_of(q, anc)
        prep_noisy = prep_noisy or noise.error_for("x") is not None
        k += 1
    if k >= len(data) or data[k].name != "h" or data[k].qubits != (anc,):
        raise NotImplementedError("expected H on the ancilla after state preparation")
    k += 1
    if k >= len(data) or data[k].name != "cz" or anc not in data[k].qubits:
        raise NotImplementedError("expected CZ(probe, ancilla)")
    pq = [q for q in data[k].qubits if q != anc][0]
    probe = _site_of(pq, anc)
    k += 1
    if (len(data) - k < 3 or data[-3].name != "cz" or set(data[-3].qubits) != {pq, anc}
            or data[-2].name != "h" or data[-2].qubits != (anc,)):
        raise NotImplementedError("expected CZ(probe, ancilla), H, measure at the end")
    body = data[k:-3]
    for ins in body:
        if anc in ins.qubits:
            raise NotImplementedError("gates on the ancilla inside the evolution")
        if ins.name not in _KICK_GATES | _DIAG_GATES:
            raise NotImplementedError(f"gate {ins.name} inside the evolution")

    # split the body into kick runs and diagonal chunks of (2L-1) gates
    n_diag = (L - 1) + L
    runs = []
    cur = None
    for ins in body:
        typ = "K" if ins.name in _KICK_GATES else "D"
        if cur is None or cur[0] != typ:
            cur = (typ, [])
            runs.append(cur)
        cur[1].append(ins)
    # forward period = K then D (fast.py:111-121); inverse = D then K (fast.py:140-143).
    # A forward D directly followed by another D starts the echo.
    fwd_kicks, fwd_diag, inv_kicks, inv_diag = [], [], [], []
    toks = []
    for typ, gs in runs:
        if typ == "K":
            toks.append(("K", gs))
        else:
            if len(gs) % n_diag:
                raise NotImplementedError("diagonal layer does not match RZZ/RZ of a period")
            toks.extend(("D", gs[c:c + n_diag]) for c in range(0, len(gs), n_diag))
    i = 0
    while i + 1 < len(toks) and toks[i][0] == "K" and toks[i + 1][0] == "D":
        fwd_kicks.append(toks[i][1])
        fwd_diag.append(toks[i + 1][1])
        i += 2
    while i < len(toks):
        if toks[i][0] != "D" or i + 1 >= len(toks) or toks[i + 1][0] != "K":
            raise NotImplementedError("evolution is not U_F^t [U_F^-t]")
        inv_diag.append(toks[i][1])
        inv_kicks.append(toks[i + 1][1])
        i += 2
    nf, ni = len(fwd_kicks), len(inv_kicks)
    if ni not in (0, nf):
        raise NotImplementedError("echo must invert every forward period")

    def diag_angles(chunk, sign):
        hs = np.zeros(L)
        ph = np.zeros(max(L - 1, 1))
        for ins in chunk:
            if ins.name == "rz":
                hs[_site_of(ins.qubits[0], anc)] += sign * ins.params[0]
            else:
                a, b = sorted(_site_of(q, anc) for q in ins.qubits)
                if b != a + 1:
                    raise NotImplementedError("RZZ on a non-nearest-neighbour bond")
                ph[a] += sign * ins.params[0]
        return hs, ph

    if nf:
        hs, ph = diag_angles(fwd_diag[0], 1.0)
        for ch in fwd_diag[1:]:
            h2, p2 = diag_angles(ch, 1.0)
            if not (np.allclose(h2, hs, atol=1e-12) and np.allclose(p2, ph, atol=1e-12)):
                raise NotImplementedError("disorder changes between periods")
        for ch in inv_diag:
            h2, p2 = diag_angles(ch, -1.0)
            if not (np.allclose(h2, hs, atol=1e-12) and np.allclose(p2, ph, atol=1e-12)):
                raise NotImplementedError("echo diagonal is not the inverse of the forward one")
    else:
        hs, ph = np.zeros(L), np.zeros(max(L - 1, 1))

    def site_gates(kick_run):
        per = [[] for _ in range(L)]
        for ins in kick_run:
            m = rx_m(ins.params[0]) if ins.name == "rx" else ry_m(ins.params[0])
            per[_site_of(ins.qubits[0], anc)].append(m)
        return per

    n_sub = None
    rows = []
    for run in fwd_kicks:
        per = site_gates(run)
        counts = {len(g) for g in per}
        if len(counts) != 1 or 0 in counts:
            raise NotImplementedError("every site must be kicked the same number of times")
        c = counts.pop()
        if n_sub is None:
            n_sub = c
        elif c != n_sub:
            raise NotImplementedError("kick sub-gate count changes between periods")
        rows.append(per)
    n_sub = n_sub or 1
    kick = np.zeros((max(1, nf), L, n_sub, 8))
    for s, per in enumerate(rows):
        for site in range(L):
            for q, m in enumerate(per[site]):
                kick[s, site, q] = matrix_to_row(m)
    if nf == 0:
        for site in range(L):
            for q in range(n_sub):
                kick[0, site, q] = matrix_to_row(np.eye(2))
    # the echo must replay the forward kicks inverted, periods in reverse order
    for e, run in enumerate(inv_kicks):
        s = nf - 1 - e
        per = site_gates(run)
        for site in range(L):
            fw = rows[s][site]
            if len(per[site]) != len(fw):
                raise NotImplementedError("echo kick does not invert the forward kick")
            prod_f = np.eye(2, dtype=complex)
            for m in fw:
                prod_f = m @ prod_f
            prod_i = np.eye(2, dtype=complex)
            for m in per[site]:
                prod_i = m @ prod_i
            if not np.allclose(prod_i @ prod_f, np.eye(2), atol=1e-10):
                raise NotImplementedError("echo kick does not invert the forward kick")

    kick_noisy = any(noise.error_for(g.name) is not None for run in fwd_kicks + inv_kicks
                     for g in run)
    n_anc = 6 if noise.error_for("h") is not None else 0
    return FoldedCircuit(L=L, n_fwd=nf, echo=ni > 0, probe=probe, init_mask=init,
                         hs=hs[None, :], phis=ph[None, : max(L - 1, 1)], kick=kick,
                         kick_noisy=kick_noisy, n_anc_noisy=n_anc, prep_noisy=prep_noisy)


def _noise_p(noise: NoiseModel | None) -> float:
    if noise is None or noise.is_ideal():
        return 0.0
    ps = {e.p for e in noise._errors.values()}
    kinds = {e.kind for e in noise._errors.values()}
    if kinds != {"depolarizing"} or len(ps) != 1:
        raise NotImplementedError("only one common depolarizing_error(p, 1) is supported")
    return ps.pop()


_ENGINES: dict[int, DtcEngine] = {}


def get_engine(device: int = 0) -> DtcEngine:
    if device not in _ENGINES:
        _ENGINES[device] = DtcEngine(device)
    return _ENGINES[device]


class DtcResult:
    def __init__(self, counts_list, circuits, expectations):
        self._counts = counts_list
        self._circuits = circuits
        self.expectations = expectations  # exact/trajectory-mean <Z_anc> per circuit
        self.success = True

    def get_counts(self, experiment=None):
        if experiment is None:
            return self._counts[0] if len(self._counts) == 1 else list(self._counts)
        if isinstance(experiment, int):
            return self._counts[experiment]
        for c, circ in zip(self._counts, self._circuits):
            if circ is experiment:
                return c
        raise KeyError("circuit not part of this result")


class DtcJob:
    def __init__(self, result: DtcResult):
        self._result = result

    def result(self):
        return self._result

    def status(self):
        return "DONE"


class DtcSimulator:
    """AerSimulator-shaped backend running folded DTC circuits on gfx950."""

    name = "aer_simulator"

    def __init__(self, noise_model: NoiseModel | None = None, device="GPU", seed_simulator=None,
                 device_index: int = 0, **options):
        if str(device).upper() != "GPU":
            raise NotImplementedError("the DTC engine runs on the MI355X only (device='GPU')")
        self.noise_model = noise_model
        self.options = dict(options)
        self.seed_simulator = seed_simulator
        self.device_index = device_index
        self._calls = 0

    def run(self, circuits, shots: int = 1024, seed_simulator=None, **kw) -> DtcJob:
        single = isinstance(circuits, QuantumCircuit)
        circs = [circuits] if single else list(circuits)
        seed = seed_simulator if seed_simulator is not None else self.seed_simulator
        if seed is None:
            seed = int(np.random.SeedSequence().generate_state(1, np.uint64)[0])
        cal = getattr(self.noise_model, "device_calibration", None)
        p = 0.0 if cal is not None else _noise_p(self.noise_model)
        eng = get_engine(self.device_index)
        counts, expv = [], []
        for ci, circ in enumerate(circs):
            if cal is not None:
                a = _run_device(eng, circ, cal, shots, seed + 7919 * (self._calls + ci))
                rng = np.random.default_rng([seed, self._calls, ci])
                n0 = int(rng.binomial(shots, float(np.clip((1.0 + a) / 2.0, 0.0, 1.0))))
                c = {}
                if n0:
                    c["0"] = n0
                if shots - n0:
                    c["1"] = shots - n0
                counts.append(c)
                expv.append(a)
                continue
            f = fold_circuit(circ, self.noise_model)
            # kicks and X preps both transpile to u3: one noise probability for both
            pk = p if (f.kick_noisy or f.prep_noisy) else 0.0
            T = f.n_fwd + 1
            spec = SweepSpec(L=f.L, T=T, hs=f.hs, phis=f.phis, kick=f.kick,
                             noise_prob=pk, use_noise=1, probe_site=f.probe,
                             init_mask_value=f.init_mask)
            n_traj = shots if pk > 0 else 1
            out = _run_single(eng, spec, f, n_traj, seed + 7919 * (self._calls + ci), p)
            a = out  # per-trajectory ancilla expectations at t = n_fwd
            rng = np.random.default_rng([seed, self._calls, ci])
            if n_traj == 1:
                n0 = int(rng.binomial(shots, (1.0 + a[0]) / 2.0))
            else:
                n0 = int(np.sum(rng.random(shots) < (1.0 + a) / 2.0))
            c = {}
            if n0:
                c["0"] = n0
            if shots - n0:
                c["1"] = shots - n0
            counts.append(c)
            expv.append(float(np.mean(a)))
        self._calls += len(circs)
        return DtcJob(DtcResult(counts, circs, expv))


def _run_single(eng: DtcEngine, spec: SweepSpec, f: FoldedCircuit, n_traj: int, seed: int,
                p_anc: float):
    """Per-trajectory ancilla expectation of one folded circuit."""
    from . import _capi
    import ctypes

    T = spec.T
    pr = eng._problem(spec, want_fwd=not f.echo, want_echo=f.echo, batch=0, t_first=T - 1)
    nz = _capi.DtcNoise()
    nz.p = spec.p
    nz.n_anc = 0
    fwd = np.zeros((1, n_traj, T))
    echo = np.zeros((1, n_traj, T))
    _capi.check(eng._lib.dtc_autocorr(
        eng._ctx, ctypes.byref(pr), ctypes.byref(nz), ctypes.c_uint64(seed & (2**64 - 1)),
        ctypes.c_int64(0), ctypes.c_int32(n_traj), _capi.as_dptr(fwd if not f.echo else None),
        _capi.as_dptr(echo if f.echo else None), None))
    a = (echo if f.echo else fwd)[0, :, T - 1]
    return a * (1.0 - p_anc) ** f.n_anc_noisy


def _run_device(eng: DtcEngine, circ, cal, shots: int, seed: int) -> float:
    """Trajectory-mean read-out expectation of one folded circuit under the
    calibration's device-like noise (dtc_autocorr_device)."""
    f = fold_circuit(circ, None)
    T = f.n_fwd + 1
    dev = cal.device_noise(f.L)  # every kick is a physical (noisy) gate on the device
    spec = SweepSpec(L=f.L, T=T, hs=f.hs, phis=f.phis, kick=f.kick, probe_site=f.probe,
                     init_mask_value=f.init_mask, device=dev)
    out = eng.autocorr(spec, max(1, shots), seed=seed & (2**64 - 1),
                       want_fwd=not f.echo, want_echo=f.echo, t_first=T - 1)
    a = (out["echo"] if f.echo else out["fwd"])[0, :, T - 1]
    return float(np.mean(a))


AerSimulator = DtcSimulator
