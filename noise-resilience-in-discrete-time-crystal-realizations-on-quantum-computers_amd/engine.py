"""Host-side handle on the HIP engine (one ``dtc_ctx`` per device).

This is the layer the reference's drivers reach through
``AerSimulator(...).run(circ, shots).result().get_counts()`` (fast.py:156,
211-212); here the whole t-sweep of a disorder instance is one call, see
``include/dtc.h``.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import _capi
from .kicks import kick_table, n_sub_of

N_ANCILLA_NOISY_GATES = 6  # H, CZ=u2.cx.u2 (x2), H on the ancilla -> six noisy u2


@dataclass
class SweepSpec:
    """Everything that defines one autocorrelator sweep (fast.py argparse +
    disorder).  ``hs``: [n_inst][L], ``phis``: [n_inst][L-1]."""

    L: int
    T: int
    hs: np.ndarray
    phis: np.ndarray
    g: float | list = 0.97
    polarization: str = "x"
    circular_frequency: float = 1.0
    initial_state: str = "vacuum"
    noise_prob: float = 0.05
    use_noise: int = 1
    t_offset: int = 0
    probe_site: int | None = None
    kick: np.ndarray | None = field(default=None, repr=False)
    init_mask_value: int | None = None   # explicit Z-basis prep (overrides initial_state)
    device: object | None = field(default=None, repr=False)  # DeviceNoise (use_fakebackend=1)

    def __post_init__(self):
        self.hs = np.ascontiguousarray(np.atleast_2d(self.hs)[:, : self.L], dtype=np.float64)
        ph = np.atleast_2d(self.phis)
        self.phis = np.ascontiguousarray(ph[:, : max(self.L - 1, 0)], dtype=np.float64)
        if self.L == 1:
            self.phis = np.zeros((self.hs.shape[0], 1))
        if self.probe_site is None:
            self.probe_site = int(self.L / 2)  # fast.py:221
        if self.kick is None:
            self.kick = kick_table(self.L, self.n_periods, self.g, self.polarization,
                                   self.circular_frequency)
        self.kick = np.ascontiguousarray(self.kick, dtype=np.float64)

    @property
    def n_inst(self) -> int:
        return self.hs.shape[0]

    @property
    def n_periods(self) -> int:
        return max(1, self.T - 1 + self.t_offset)

    @property
    def n_sub(self) -> int:
        return self.kick.shape[2]

    @property
    def p(self) -> float:
        return float(self.noise_prob) if self.use_noise else 0.0

    @property
    def init_mask(self) -> int:
        if self.init_mask_value is not None:
            return int(self.init_mask_value)
        return init_mask(self.L, self.initial_state)


def init_mask(L: int, initial_state: str) -> int:
    """fast.py:127-130: ``neel`` = X on circuit qubits 2, 4, ... (sites 1, 3, ...)."""
    if initial_state == "vacuum":
        return 0
    if initial_state == "neel":
        m = 0
        for q in range(1, L + 1):
            if q % 2 == 0:
                m |= 1 << (q - 1)
        return m
    raise ValueError(f"initial_state must be 'vacuum' or 'neel', got {initial_state!r}")


def energy_init_mask(L: int, initial_state: str) -> int:
    """The energy scripts' preparation (autocorr-delta-a-single-qiskit-fast-energy.py:137-141,
    the same loop in every ``-energy*.py``): ``for i in range(1, L+1): if i % 2 == 0:
    circ.x(i)`` on ``QuantumCircuit(L)`` -- L qubits, no ancilla, so qubit i IS site i.
    For odd L that flips sites 2, 4, ..., L-1; for even L the loop reaches
    ``circ.x(L)`` on an L-qubit circuit and qiskit raises (index out of range), so
    this raises too.  (The autocorrelator's ``init_mask`` differs: there qubit 0
    is the ancilla and circuit qubit i is site i-1.)"""
    if initial_state == "vacuum":
        return 0
    if initial_state != "neel":
        raise ValueError(f"initial_state must be 'vacuum' or 'neel', got {initial_state!r}")
    m = 0
    for i in range(1, L + 1):
        if i % 2 == 0:
            if i >= L:
                raise ValueError(
                    f"neel preparation of the {L}-qubit energy circuit applies X to qubit {i}, "
                    f"out of range(0, {L}) (the reference's circ.x({i}) raises for even L)")
            m |= 1 << i
    return m


class DtcEngine:
    """Owns one device context of libdtc_hip.so."""

    def __init__(self, device: int = 0):
        self._lib = _capi.load_library()
        ctx = ctypes.c_void_p()
        _capi.check(self._lib.dtc_open(int(device), ctypes.byref(ctx)))
        self._ctx = ctx
        self.device = device

    def close(self):
        if getattr(self, "_ctx", None) is not None and self._ctx.value:
            self._lib.dtc_close(self._ctx)
            self._ctx = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- structs -------------------------------------------------------
    @staticmethod
    def _problem(spec: SweepSpec, want_fwd=True, want_echo=True, batch=0, t_first=0):
        pr = _capi.DtcProblem()
        pr.L = spec.L
        pr.T = spec.T
        pr.n_inst = spec.n_inst
        pr.probe_site = spec.probe_site
        pr.t_offset = spec.t_offset
        pr.n_sub = spec.n_sub
        pr.init_mask = spec.init_mask
        pr.h = _capi.as_dptr(spec.hs)
        pr.phi = _capi.as_dptr(spec.phis)
        pr.kick = _capi.as_dptr(spec.kick)
        pr.want_fwd = int(bool(want_fwd))
        pr.want_echo = int(bool(want_echo))
        pr.batch = int(batch)
        pr.t_first = int(t_first)
        return pr

    @staticmethod
    def _noise(spec: SweepSpec):
        nz = _capi.DtcNoise()
        nz.p = spec.p
        nz.n_anc = N_ANCILLA_NOISY_GATES
        return nz

    # -- API -------------------------------------------------------------
    def autocorr(self, spec: SweepSpec, n_traj: int, seed: int = 0x5EED0001,
                 traj_offset: int = 0, want_fwd: bool = True, want_echo: bool = True,
                 want_zsite: bool = False, batch: int = 0, t_first: int = 0):
        """Per-trajectory ancilla expectations.

        Returns dict with ``fwd``/``echo`` of shape [n_inst][n_traj][T] and
        optionally ``zsite`` [n_inst][n_traj][T][L] (forward <Z_i>(t)).
        """
        n_inst, T, L = spec.n_inst, spec.T, spec.L
        fwd = np.zeros((n_inst, n_traj, T)) if want_fwd else None
        echo = np.zeros((n_inst, n_traj, T)) if want_echo else None
        zs = np.zeros((n_inst, n_traj, T, L)) if want_zsite else None
        pr = self._problem(spec, want_fwd, want_echo, batch, t_first)
        if spec.device is not None:
            # device-like noise (include/dtc.h dtc_device_noise); spec.noise_prob unused
            if spec.device.L != spec.L:
                raise ValueError("device noise has a different number of sites")
            dv = _capi.device_struct(spec.device)
            _capi.check(self._lib.dtc_autocorr_device(
                self._ctx, ctypes.byref(pr), ctypes.byref(dv), ctypes.c_uint64(seed),
                ctypes.c_int64(traj_offset), ctypes.c_int32(n_traj), _capi.as_dptr(fwd),
                _capi.as_dptr(echo), _capi.as_dptr(zs)))
        else:
            nz = self._noise(spec)
            _capi.check(self._lib.dtc_autocorr(
                self._ctx, ctypes.byref(pr), ctypes.byref(nz), ctypes.c_uint64(seed),
                ctypes.c_int64(traj_offset), ctypes.c_int32(n_traj), _capi.as_dptr(fwd),
                _capi.as_dptr(echo), _capi.as_dptr(zs)))
        out = {}
        if want_fwd:
            out["fwd"] = fwd
        if want_echo:
            out["echo"] = echo
        if want_zsite:
            out["zsite"] = zs
        return out

    # -- forward prefix cache (dtc_prefix_*; user: control.optimize_g) ------
    def prefix_build(self, spec: SweepSpec, n_traj: int, n_periods: int,
                     seed: int = 0x5EED0001, traj_offset: int = 0):
        """Keep every trajectory's state after periods 1..n_periods on the device."""
        pr = self._problem(spec)
        dv = _capi.device_struct(spec.device) if spec.device is not None else None
        _capi.check(self._lib.dtc_prefix_build(
            self._ctx, ctypes.byref(pr), ctypes.byref(self._noise(spec)),
            ctypes.byref(dv) if dv is not None else None, ctypes.c_uint64(seed),
            ctypes.c_int64(traj_offset), ctypes.c_int32(n_traj), ctypes.c_int32(n_periods)))

    def autocorr_prefixed(self, spec: SweepSpec, n_traj: int, seed: int = 0x5EED0001,
                          traj_offset: int = 0, want_fwd: bool = True, want_echo: bool = True,
                          t_first: int = 0, batch: int = 0):
        """``autocorr`` continuing from the prefix (periods after it and every
        echo drawn from ``seed``); same outputs without ``zsite``."""
        n_inst, T = spec.n_inst, spec.T
        fwd = np.zeros((n_inst, n_traj, T)) if want_fwd else None
        echo = np.zeros((n_inst, n_traj, T)) if want_echo else None
        pr = self._problem(spec, want_fwd, want_echo, batch, t_first)
        dv = _capi.device_struct(spec.device) if spec.device is not None else None
        _capi.check(self._lib.dtc_autocorr_prefixed(
            self._ctx, ctypes.byref(pr), ctypes.byref(self._noise(spec)),
            ctypes.byref(dv) if dv is not None else None, ctypes.c_uint64(seed),
            ctypes.c_int64(traj_offset), ctypes.c_int32(n_traj), _capi.as_dptr(fwd),
            _capi.as_dptr(echo)))
        out = {}
        if want_fwd:
            out["fwd"] = fwd
        if want_echo:
            out["echo"] = echo
        return out

    def prefix_release(self):
        _capi.check(self._lib.dtc_prefix_release(self._ctx))

    def apply_periods(self, spec: SweepSpec, state: np.ndarray, first_period: int,
                      n_periods: int, inverse: bool = False, inst: int = 0, traj: int = 0,
                      stream: int = 0, seed: int = 0x5EED0001):
        """Apply periods to a host statevector (complex128 [2^L]); returns
        ``(new_state, [norm, <Z_0>, ..., <Z_{L-1}>])``."""
        psi = np.ascontiguousarray(state, dtype=np.complex128).copy()
        if psi.shape != (1 << spec.L,):
            raise ValueError("state must have 2^L amplitudes")
        buf = psi.view(np.float64)
        z = np.zeros(1 + spec.L)
        pr = self._problem(spec)
        nz = self._noise(spec)
        _capi.check(self._lib.dtc_apply_periods(
            self._ctx, ctypes.byref(pr), ctypes.byref(nz), ctypes.c_uint64(seed),
            ctypes.c_int32(inst), ctypes.c_int64(traj), ctypes.c_uint32(stream),
            ctypes.c_int32(first_period), ctypes.c_int32(n_periods),
            ctypes.c_int32(int(inverse)), _capi.as_dptr(buf), _capi.as_dptr(z)))
        return psi, z

    def energy(self, spec: SweepSpec, n_traj: int, seed: int = 0x5EED0001,
               traj_offset: int = 0, batch: int = 0):
        """Per-trajectory energy observables of the forward sweep (dtc_energy,
        or dtc_energy_device when ``spec.device`` is set: Kraus-weighted
        expectations, read-out error not applied): ``z`` [n_inst][n_traj][T][L],
        ``zz`` [..][L-1], ``x`` [..][L]."""
        n_inst, T, L = spec.n_inst, spec.T, spec.L
        z = np.zeros((n_inst, n_traj, T, L))
        zz = np.zeros((n_inst, n_traj, T, max(L - 1, 0)))
        x = np.zeros((n_inst, n_traj, T, L))
        pr = self._problem(spec, True, False, batch, 0)
        outs = (_capi.as_dptr(z), _capi.as_dptr(zz) if L > 1 else None, _capi.as_dptr(x))
        if spec.device is not None:
            if spec.device.L != spec.L:
                raise ValueError("device noise has a different number of sites")
            dv = _capi.device_struct(spec.device)
            _capi.check(self._lib.dtc_energy_device(
                self._ctx, ctypes.byref(pr), ctypes.byref(dv), ctypes.c_uint64(seed),
                ctypes.c_int64(traj_offset), ctypes.c_int32(n_traj), *outs))
        else:
            _capi.check(self._lib.dtc_energy(
                self._ctx, ctypes.byref(pr), ctypes.byref(self._noise(spec)),
                ctypes.c_uint64(seed), ctypes.c_int64(traj_offset), ctypes.c_int32(n_traj),
                *outs))
        return {"z": z, "zz": zz, "x": x}

    def energy_sums(self, spec: SweepSpec, n_traj: int, seed: int = 0x5EED0001,
                    traj_offset: int = 0, batch: int = 0):
        """``energy``'s observables summed over each instance's ``n_traj``
        trajectories on the device (dtc_energy_sums; device-like noise when
        ``spec.device`` is set): ``z`` [n_inst][T][L], ``zz`` [..][L-1], ``x``
        [..][L].  Divide by ``n_traj`` for the estimator's means."""
        n_inst, T, L = spec.n_inst, spec.T, spec.L
        z = np.zeros((n_inst, T, L))
        zz = np.zeros((n_inst, T, max(L - 1, 0)))
        x = np.zeros((n_inst, T, L))
        pr = self._problem(spec, True, False, batch, 0)
        dv = None
        if spec.device is not None:
            if spec.device.L != spec.L:
                raise ValueError("device noise has a different number of sites")
            dv = _capi.device_struct(spec.device)
        _capi.check(self._lib.dtc_energy_sums(
            self._ctx, ctypes.byref(pr), ctypes.byref(self._noise(spec)),
            ctypes.byref(dv) if dv is not None else None, ctypes.c_uint64(seed),
            ctypes.c_int64(traj_offset), ctypes.c_int32(n_traj), _capi.as_dptr(z),
            _capi.as_dptr(zz) if L > 1 else None, _capi.as_dptr(x)))
        return {"z": z, "zz": zz, "x": x}

    # -- sharded state (dtc_shard_*; driver: sharded.py) ----------------
    def shard_set_basis(self, spec: SweepSpec, shard, state_ptr: int, seed: int = 0x5EED0001,
                        traj: int = 0):
        """Prepare the (noisy-prep) product state in device buffer ``state_ptr``."""
        _capi.check(self._lib.dtc_shard_set_basis(
            self._ctx, ctypes.byref(self._problem(spec)), ctypes.byref(self._noise(spec)),
            ctypes.byref(shard), ctypes.c_uint64(seed), ctypes.c_int64(traj),
            ctypes.c_void_p(state_ptr)))

    def shard_step(self, spec: SweepSpec, shard, period: int, pre_mask: int, diag: bool,
                   post_mask: int, src_ptr: int, dst_ptr: int, want_obs: bool = False,
                   seed: int = 0x5EED0001, traj: int = 0, inst: int = 0):
        """dst = K_{period+1}[post] . D^diag . K_period[pre] . src on every shard held;
        returns obs [n_shards][1 + n_local] (or None)."""
        obs = np.zeros((shard.n_shards, 1 + shard.n_local)) if want_obs else None
        _capi.check(self._lib.dtc_shard_step(
            self._ctx, ctypes.byref(self._problem(spec)), ctypes.byref(self._noise(spec)),
            ctypes.byref(shard), ctypes.c_uint64(seed), ctypes.c_int64(traj),
            ctypes.c_int32(inst), ctypes.c_int32(period), ctypes.c_uint64(pre_mask),
            ctypes.c_int32(int(bool(diag))), ctypes.c_uint64(post_mask),
            ctypes.c_void_p(src_ptr), ctypes.c_void_p(dst_ptr), _capi.as_dptr(obs)))
        return obs

    def shard_step_async(self, spec: SweepSpec, shard, period: int, pre_mask: int, diag: bool,
                         post_mask: int, src_ptr: int, dst_ptr: int, obs_ptr: int | None = None,
                         seed: int = 0x5EED0001, traj: int = 0, inst: int = 0):
        """shard_step enqueued on the engine stream without waiting; obs_ptr
        (device, [n_shards][1 + n_local] doubles) receives the observables."""
        _capi.check(self._lib.dtc_shard_step_async(
            self._ctx, ctypes.byref(self._problem(spec)), ctypes.byref(self._noise(spec)),
            ctypes.byref(shard), ctypes.c_uint64(seed), ctypes.c_int64(traj),
            ctypes.c_int32(inst), ctypes.c_int32(period), ctypes.c_uint64(pre_mask),
            ctypes.c_int32(int(bool(diag))), ctypes.c_uint64(post_mask),
            ctypes.c_void_p(src_ptr), ctypes.c_void_p(dst_ptr),
            ctypes.c_void_p(obs_ptr) if obs_ptr else None))

    def shard_kick_slice(self, spec: SweepSpec, shard, period: int, pre_mask: int,
                         chunk_bits: int, slice_bits: int, slice_: int, state_ptr: int,
                         seed: int = 0x5EED0001, traj: int = 0):
        """K_period on the local bits pre_mask of slice `slice_` of every chunk
        (top chunk_bits local bits; the next slice_bits number the slices) of
        every shard held, in place, asynchronously (one launch)."""
        _capi.check(self._lib.dtc_shard_kick_slice(
            self._ctx, ctypes.byref(self._problem(spec)), ctypes.byref(self._noise(spec)),
            ctypes.byref(shard), ctypes.c_uint64(seed), ctypes.c_int64(traj),
            ctypes.c_int32(period), ctypes.c_uint64(pre_mask), ctypes.c_int32(chunk_bits),
            ctypes.c_int32(slice_bits), ctypes.c_int32(slice_), ctypes.c_void_p(state_ptr)))

    def release_buffers(self, drop_prefix: bool = True):
        """Free the engine's batch work buffers (dtc_release_buffers) and, by
        default, the forward prefix (dtc_prefix_release) -- all the engine's
        large device memory, e.g. before one 256 GiB sharded state; the next
        call re-allocates what it needs."""
        if drop_prefix:
            _capi.check(self._lib.dtc_prefix_release(self._ctx))
        _capi.check(self._lib.dtc_release_buffers(self._ctx))

    def shard_exchange_slice(self, shard, slice_bits: int, slice_: int, state_ptr: int):
        """Virtual ranks (every shard in ``state_ptr``): the all-to-all of slice
        ``slice_`` in place -- piece (shard r, chunk c) <-> (shard c, chunk r) --
        asynchronously on the engine stream (one launch)."""
        _capi.check(self._lib.dtc_shard_exchange_slice(
            self._ctx, ctypes.byref(shard), ctypes.c_int32(slice_bits), ctypes.c_int32(slice_),
            ctypes.c_void_p(state_ptr)))

    def shard_kick_exchange_slice(self, spec: SweepSpec, shard, period: int, pre_mask: int,
                                  slice_bits: int, slice_: int, state_ptr: int,
                                  seed: int = 0x5EED0001, traj: int = 0):
        """Virtual ranks: ``shard_kick_slice`` (chunk bits = n_global) and
        ``shard_exchange_slice`` of slice ``slice_`` as one step -- the last
        site group's kick pass stores each piece at its partner's place
        (dtc_shard_kick_exchange_slice), so the exchange moves no bytes of its
        own."""
        _capi.check(self._lib.dtc_shard_kick_exchange_slice(
            self._ctx, ctypes.byref(self._problem(spec)), ctypes.byref(self._noise(spec)),
            ctypes.byref(shard), ctypes.c_uint64(seed), ctypes.c_int64(traj),
            ctypes.c_int32(period), ctypes.c_uint64(pre_mask), ctypes.c_int32(slice_bits),
            ctypes.c_int32(slice_), ctypes.c_void_p(state_ptr)))

    def stream_handle(self) -> int:
        """The engine's hipStream_t (for torch.cuda.ExternalStream)."""
        h = ctypes.c_void_p()
        _capi.check(self._lib.dtc_get_stream(self._ctx, ctypes.byref(h)))
        return int(h.value or 0)

    def synchronize(self):
        _capi.check(self._lib.dtc_synchronize(self._ctx))

    # -- profiling -------------------------------------------------------
    def set_profiling(self, on: bool):
        _capi.check(self._lib.dtc_set_profiling(self._ctx, int(on)))

    def reset_stats(self):
        _capi.check(self._lib.dtc_reset_stats(self._ctx))

    def kernel_stats(self):
        out = {}
        for k in range(_capi.KERNEL_KINDS):
            n = ctypes.c_int64()
            ms = ctypes.c_double()
            by = ctypes.c_double()
            _capi.check(self._lib.dtc_kernel_stats(self._ctx, k, ctypes.byref(n),
                                                   ctypes.byref(ms), ctypes.byref(by)))
            out[k] = {"launches": n.value, "total_ms": ms.value, "bytes": by.value}
        return out

    def lightcone_counts(self):
        """Light-cone ends launched since the engine opened, by kernel
        (dtc_lightcone_counts): 8-site window, 10-site generic, 10-site C2 form,
        12-site C2 form."""
        c = (ctypes.c_int64 * 4)()
        _capi.check(self._lib.dtc_lightcone_counts(self._ctx, c))
        return {"lc8": c[0], "lcw": c[1], "lcw2": c[2], "lcw3": c[3]}

    def schedule_counts(self):
        """Batch schedules built since the engine opened (dtc_schedule_counts):
        echo chains folded into a dual pass, device-noise batches whose forward
        ran a layer ahead, device-noise batches run with K-D forward passes
        (a chain did not fold, or DTC_NO_RUNAHEAD=1), and batches run with the
        13 / 7 site split of L = 20."""
        c = (ctypes.c_int64 * 4)()
        _capi.check(self._lib.dtc_schedule_counts(self._ctx, c))
        return {"folded": c[0], "device_runahead": c[1], "device_kd": c[2], "split13": c[3]}

    def device_info(self):
        name = ctypes.create_string_buffer(256)
        ncu = ctypes.c_int32()
        mem = ctypes.c_double()
        _capi.check(self._lib.dtc_device_info(self._ctx, name, 256, ctypes.byref(ncu),
                                              ctypes.byref(mem)))
        return {"name": name.value.decode(), "n_cu": ncu.value, "hbm_bytes": mem.value}


def spec_n_sub(polarization: str) -> int:
    return n_sub_of(polarization)
