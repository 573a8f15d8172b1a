"""ctypes wrapper of oracle/liboracle.so (the C restatement in dtc_oracle.c).

TEST INFRASTRUCTURE ONLY — used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
LIB_PATH_V3 = os.path.join(_HERE, "liboracle_v3.so")  # -march=x86-64-v3 build (Makefile)
_V3_FLAGS = {"avx", "avx2", "bmi1", "bmi2", "f16c", "fma", "movbe", "abm"}


def _host_has_v3() -> bool:
    """The x86-64-v3 feature set in /proc/cpuinfo (else the portable build)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    return _V3_FLAGS <= set(line.split(":", 1)[1].split())
    except OSError:
        pass
    return False


def lib_path() -> str:
    """The build this host runs: the x86-64-v3 one when present and supported."""
    if os.path.exists(LIB_PATH_V3) and _host_has_v3():
        return LIB_PATH_V3
    return LIB_PATH

_dp = ctypes.POINTER(ctypes.c_double)


class OrcProblem(ctypes.Structure):
    _fields_ = [
        ("L", ctypes.c_int32), ("T", ctypes.c_int32), ("n_inst", ctypes.c_int32),
        ("probe_site", ctypes.c_int32), ("t_offset", ctypes.c_int32),
        ("n_sub", ctypes.c_int32), ("init_mask", ctypes.c_uint64), ("h", _dp),
        ("phi", _dp), ("kick", _dp), ("want_fwd", ctypes.c_int32),
        ("want_echo", ctypes.c_int32), ("batch", ctypes.c_int32),
        ("t_first", ctypes.c_int32),
    ]


class OrcNoise(ctypes.Structure):
    _fields_ = [("p", ctypes.c_double), ("n_anc", ctypes.c_int32),
                ("reserved", ctypes.c_int32)]


class OrcDeviceNoise(ctypes.Structure):
    _fields_ = [("p_gate", _dp), ("t1_us", _dp), ("t2_us", _dp), ("gate_ns", ctypes.c_double),
                ("anc_factor", ctypes.c_double), ("readout_p01", ctypes.c_double),
                ("readout_p10", ctypes.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        path = lib_path()
        if not os.path.exists(path):
            raise RuntimeError(f"oracle not built: {path} (run `make`)")
        _lib = ctypes.CDLL(path)
        _lib.orc_autocorr.argtypes = [ctypes.POINTER(OrcProblem), ctypes.POINTER(OrcNoise),
                                      ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, _dp, _dp,
                                      _dp, ctypes.c_int32]
        _lib.orc_apply_periods.argtypes = [ctypes.POINTER(OrcProblem), ctypes.POINTER(OrcNoise),
                                           ctypes.c_uint64, ctypes.c_int32, ctypes.c_int64,
                                           ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32,
                                           ctypes.c_int32, _dp, _dp]
        _lib.orc_sample_pauli.argtypes = [ctypes.c_double, ctypes.c_uint64, ctypes.c_uint64,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32]
        _lib.orc_sample_pauli.restype = ctypes.c_int
        _lib.orc_autocorr_device.argtypes = [
            ctypes.POINTER(OrcProblem), ctypes.POINTER(OrcDeviceNoise), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_int32, _dp, _dp, _dp, ctypes.c_int32]
        _lib.orc_apply_periods_device.argtypes = [
            ctypes.POINTER(OrcProblem), ctypes.POINTER(OrcDeviceNoise), ctypes.c_uint64,
            ctypes.c_int32, ctypes.c_int64, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_int32, _dp, _dp]
        _lib.orc_init_mask.argtypes = [ctypes.POINTER(OrcProblem), ctypes.c_double,
                                       ctypes.POINTER(OrcDeviceNoise), ctypes.c_uint64,
                                       ctypes.c_int64]
        _lib.orc_init_mask.restype = ctypes.c_int64
        _lib.orc_autocorr_fused.argtypes = [ctypes.POINTER(OrcProblem), ctypes.POINTER(OrcNoise),
                                            ctypes.c_uint64, ctypes.c_int64, ctypes.c_int32, _dp,
                                            _dp, ctypes.c_int32]
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(_dp)


def _problem(spec, want_fwd=True, want_echo=True, t_first=0):
    pr = OrcProblem()
    pr.L, pr.T, pr.n_inst = spec.L, spec.T, spec.n_inst
    pr.probe_site, pr.t_offset, pr.n_sub = spec.probe_site, spec.t_offset, spec.n_sub
    pr.init_mask = spec.init_mask
    pr.h, pr.phi, pr.kick = _ptr(spec.hs), _ptr(spec.phis), _ptr(spec.kick)
    pr.want_fwd, pr.want_echo = int(want_fwd), int(want_echo)
    pr.t_first = int(t_first)
    return pr


def _noise(spec, n_anc=6):
    nz = OrcNoise()
    nz.p = spec.p
    nz.n_anc = n_anc
    return nz


def _device(spec):
    """OrcDeviceNoise of spec.device (its arrays stay owned by spec.device), or None."""
    dev = getattr(spec, "device", None)
    if dev is None:
        return None
    dv = OrcDeviceNoise()
    dv.p_gate, dv.t1_us, dv.t2_us = _ptr(dev.p_gate), _ptr(dev.t1_us), _ptr(dev.t2_us)
    dv.gate_ns, dv.anc_factor = dev.gate_ns, dev.anc_factor
    dv.readout_p01, dv.readout_p10 = dev.readout_p01, dev.readout_p10
    return dv


def autocorr(spec, n_traj, seed=0x5EED0001, traj_offset=0, want_fwd=True, want_echo=True,
             want_zsite=False, n_threads=0, t_first=0):
    """Same contract as DtcEngine.autocorr (per-trajectory outputs)."""
    n_inst, T, L = spec.n_inst, spec.T, spec.L
    fwd = np.zeros((n_inst, n_traj, T)) if want_fwd else None
    echo = np.zeros((n_inst, n_traj, T)) if want_echo else None
    zs = np.zeros((n_inst, n_traj, T, L)) if want_zsite else None
    dv = _device(spec)
    if dv is not None:
        rc = lib().orc_autocorr_device(ctypes.byref(_problem(spec, want_fwd, want_echo, t_first)),
                                       ctypes.byref(dv), seed, traj_offset, n_traj, _ptr(fwd),
                                       _ptr(echo), _ptr(zs), n_threads)
    else:
        rc = lib().orc_autocorr(ctypes.byref(_problem(spec, want_fwd, want_echo, t_first)),
                                ctypes.byref(_noise(spec)), seed, traj_offset, n_traj, _ptr(fwd),
                                _ptr(echo), _ptr(zs), n_threads)
    if rc != 0:
        raise RuntimeError(f"orc_autocorr failed: {rc}")
    out = {}
    if want_fwd:
        out["fwd"] = fwd
    if want_echo:
        out["echo"] = echo
    if want_zsite:
        out["zsite"] = zs
    return out


def autocorr_fused(spec, n_traj, seed=0x5EED0001, traj_offset=0, want_fwd=True,
                   want_echo=True, n_threads=0, t_first=0):
    """The period-fused CPU restatement (orc_autocorr_fused: same trajectories
    and outputs as ``autocorr``, depolarizing noise, no zsite) -- bench.py's
    CPU baseline."""
    if getattr(spec, "device", None) is not None:
        raise ValueError("autocorr_fused: depolarizing noise only")
    n_inst, T = spec.n_inst, spec.T
    fwd = np.zeros((n_inst, n_traj, T)) if want_fwd else None
    echo = np.zeros((n_inst, n_traj, T)) if want_echo else None
    rc = lib().orc_autocorr_fused(ctypes.byref(_problem(spec, want_fwd, want_echo, t_first)),
                                  ctypes.byref(_noise(spec)), seed, traj_offset, n_traj,
                                  _ptr(fwd), _ptr(echo), n_threads)
    if rc != 0:
        raise RuntimeError(f"orc_autocorr_fused failed: {rc}")
    out = {}
    if want_fwd:
        out["fwd"] = fwd
    if want_echo:
        out["echo"] = echo
    return out


def apply_periods(spec, state, first_period, n_periods, inverse=False, inst=0, traj=0,
                  stream=0, seed=0x5EED0001):
    psi = np.ascontiguousarray(state, dtype=np.complex128).copy()
    z = np.zeros(1 + spec.L)
    dv = _device(spec)
    if dv is not None:
        rc = lib().orc_apply_periods_device(ctypes.byref(_problem(spec)), ctypes.byref(dv), seed,
                                            inst, traj, stream, first_period, n_periods,
                                            int(inverse), _ptr(psi.view(np.float64)), _ptr(z))
    else:
        rc = lib().orc_apply_periods(ctypes.byref(_problem(spec)), ctypes.byref(_noise(spec)),
                                     seed, inst, traj, stream, first_period, n_periods,
                                     int(inverse), _ptr(psi.view(np.float64)), _ptr(z))
    if rc != 0:
        raise RuntimeError(f"orc_apply_periods failed: {rc}")
    return psi, z


def init_mask(spec, seed, traj):
    """Basis state after the noisy neel preparation (depolarizing or device)."""
    dv = _device(spec)
    m = lib().orc_init_mask(ctypes.byref(_problem(spec)), spec.p,
                            ctypes.byref(dv) if dv is not None else None, seed, traj)
    if m < 0:
        raise RuntimeError(f"orc_init_mask failed: {m}")
    return int(m)


def sample_pauli(p, seed, traj, stream, period, site, sub):
    return lib().orc_sample_pauli(p, seed, traj, stream, period, site, sub)
