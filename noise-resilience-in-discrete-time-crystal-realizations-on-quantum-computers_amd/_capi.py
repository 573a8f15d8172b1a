"""ctypes binding of the C ABI in ``include/dtc.h`` (``lib/libdtc_hip.so``).

The product path has exactly one implementation: the gfx950 HIP kernels in
``csrc/``.  If the shared library is missing or no gfx950 device is present
every entry point raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libdtc_hip.so")
KERNEL_KINDS = 6  # DTC_KERNEL_KINDS: lo pass, hi pass, reduce, init, final (measure-only) pass,
                  # virtual-rank exchange
ABI_VERSION = 12  # DTC_ABI_VERSION of include/dtc.h this binding matches

# Every symbol declared in include/dtc.h (checked by tests/test_capi_symbols.py).
EXPORTED_SYMBOLS = (
    "dtc_open",
    "dtc_close",
    "dtc_release_buffers",
    "dtc_last_error",
    "dtc_abi_version",
    "dtc_autocorr",
    "dtc_apply_periods",
    "dtc_set_profiling",
    "dtc_kernel_stats",
    "dtc_reset_stats",
    "dtc_lightcone_counts",
    "dtc_schedule_counts",
    "dtc_device_info",
    "dtc_shard_set_basis",
    "dtc_shard_step",
    "dtc_plan_groups",
    "dtc_energy",
    "dtc_autocorr_device",
    "dtc_energy_device",
    "dtc_energy_sums",
    "dtc_prefix_build",
    "dtc_autocorr_prefixed",
    "dtc_prefix_release",
    "dtc_shard_step_async",
    "dtc_shard_kick_slice",
    "dtc_shard_exchange_slice",
    "dtc_shard_kick_exchange_slice",
    "dtc_get_stream",
    "dtc_synchronize",
)

KERNEL_LO_PASS = 0
KERNEL_HI_PASS = 1
KERNEL_REDUCE = 2
KERNEL_INIT = 3
KERNEL_FINAL_PASS = 4
KERNEL_EXCHANGE = 5
KERNEL_NAMES = {
    KERNEL_LO_PASS: "pass_kernel<diag>  (fused RZZ+RZ diagonal + sites 0..11 kick)",
    KERNEL_HI_PASS: "pass_kernel<none>  (kick on sites >= 12)",
    KERNEL_REDUCE: "reduce_kernel",
    KERNEL_INIT: "set_basis_kernel",
    KERNEL_FINAL_PASS: "dtc_*_final / dtc_lc_final_split (measure only, no store)",
    KERNEL_EXCHANGE: "exchange_swap_kernel (virtual ranks' in-place slice exchange)",
}

_dp = ctypes.POINTER(ctypes.c_double)


class DtcProblem(ctypes.Structure):
    """Mirror of ``dtc_problem`` (include/dtc.h)."""

    _fields_ = [
        ("L", ctypes.c_int32),
        ("T", ctypes.c_int32),
        ("n_inst", ctypes.c_int32),
        ("probe_site", ctypes.c_int32),
        ("t_offset", ctypes.c_int32),
        ("n_sub", ctypes.c_int32),
        ("init_mask", ctypes.c_uint64),
        ("h", _dp),
        ("phi", _dp),
        ("kick", _dp),
        ("want_fwd", ctypes.c_int32),
        ("want_echo", ctypes.c_int32),
        ("batch", ctypes.c_int32),
        ("t_first", ctypes.c_int32),
    ]


class DtcNoise(ctypes.Structure):
    """Mirror of ``dtc_noise`` (include/dtc.h)."""

    _fields_ = [
        ("p", ctypes.c_double),
        ("n_anc", ctypes.c_int32),
        ("reserved", ctypes.c_int32),
    ]


class DtcDeviceNoise(ctypes.Structure):
    """Mirror of ``dtc_device_noise`` (include/dtc.h)."""

    _fields_ = [
        ("p_gate", _dp),
        ("t1_us", _dp),
        ("t2_us", _dp),
        ("gate_ns", ctypes.c_double),
        ("anc_factor", ctypes.c_double),
        ("readout_p01", ctypes.c_double),
        ("readout_p10", ctypes.c_double),
    ]


class DtcShard(ctypes.Structure):
    """Mirror of ``dtc_shard`` (include/dtc.h)."""

    _fields_ = [
        ("n_local", ctypes.c_int32),
        ("n_global", ctypes.c_int32),
        ("n_shards", ctypes.c_int32),
        ("first_rank", ctypes.c_int32),
        ("site_of", ctypes.c_int32 * 64),
    ]


_lib = None
_lib_lock = threading.Lock()


class DtcError(RuntimeError):
    """Raised when a C-ABI call returns a negative code."""


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load libdtc_hip.so and declare argument types.  Raises if absent."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        p = path or os.environ.get("DTC_LIB", LIB_PATH)
        if not os.path.exists(p):
            raise DtcError(
                f"HIP extension not built: {p} is missing (run `make` or "
                "`python -c 'import __graft_entry__ as g; g.build()'`)"
            )
        # One HIP runtime per process.  The PyTorch wheel ships its own
        # libamdhip64 (SONAME libamdhip64.so.7) and loads it by path; if this
        # library were loaded first it would bring in /opt/rocm's copy, and
        # torch's later device initialisation in the same process fails ("No
        # HIP GPUs are available").  Importing torch first makes this
        # library's libamdhip64.so.7 dependency resolve to the loaded copy.
        # A torch install that fails to import (ImportError, or OSError from a
        # broken wheel) only costs that ordering: the library still loads.
        try:
            import torch  # noqa: F401
        except Exception:  # noqa: BLE001
            pass
        lib = ctypes.CDLL(p)
        lib.dtc_abi_version.restype = ctypes.c_int32
        got = int(lib.dtc_abi_version())
        if got != ABI_VERSION:
            # a stale library would misread the ctypes structs below
            raise DtcError(f"{p} has C-ABI version {got}, this package expects {ABI_VERSION} "
                           "(rebuild with `make`)")
        P = ctypes.POINTER
        lib.dtc_open.argtypes = [ctypes.c_int32, P(ctypes.c_void_p)]
        lib.dtc_close.argtypes = [ctypes.c_void_p]
        lib.dtc_release_buffers.argtypes = [ctypes.c_void_p]
        lib.dtc_last_error.restype = ctypes.c_char_p
        lib.dtc_abi_version.restype = ctypes.c_int32
        lib.dtc_autocorr.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), ctypes.c_uint64, ctypes.c_int64,
            ctypes.c_int32, _dp, _dp, _dp,
        ]
        lib.dtc_apply_periods.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), ctypes.c_uint64, ctypes.c_int32,
            ctypes.c_int64, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
            _dp, _dp,
        ]
        lib.dtc_set_profiling.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        lib.dtc_kernel_stats.argtypes = [
            ctypes.c_void_p, ctypes.c_int32, P(ctypes.c_int64), _dp, _dp,
        ]
        lib.dtc_reset_stats.argtypes = [ctypes.c_void_p]
        lib.dtc_lightcone_counts.argtypes = [ctypes.c_void_p, P(ctypes.c_int64)]
        lib.dtc_schedule_counts.argtypes = [ctypes.c_void_p, P(ctypes.c_int64)]
        lib.dtc_device_info.argtypes = [
            ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32, P(ctypes.c_int32), _dp,
        ]
        lib.dtc_shard_set_basis.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), P(DtcShard), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_void_p,
        ]
        lib.dtc_shard_step.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), P(DtcShard), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int32,
            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, _dp,
        ]
        lib.dtc_shard_step_async.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), P(DtcShard), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int32,
            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
        ]
        lib.dtc_shard_kick_slice.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), P(DtcShard), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_int32, ctypes.c_void_p,
        ]
        lib.dtc_shard_exchange_slice.argtypes = [
            ctypes.c_void_p, P(DtcShard), ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p,
        ]
        lib.dtc_shard_kick_exchange_slice.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), P(DtcShard), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_int32, ctypes.c_uint64, ctypes.c_int32, ctypes.c_int32,
            ctypes.c_void_p,
        ]
        lib.dtc_get_stream.argtypes = [ctypes.c_void_p, P(ctypes.c_void_p)]
        lib.dtc_synchronize.argtypes = [ctypes.c_void_p]
        lib.dtc_energy.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), ctypes.c_uint64, ctypes.c_int64,
            ctypes.c_int32, _dp, _dp, _dp,
        ]
        lib.dtc_autocorr_device.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcDeviceNoise), ctypes.c_uint64, ctypes.c_int64,
            ctypes.c_int32, _dp, _dp, _dp,
        ]
        lib.dtc_energy_device.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcDeviceNoise), ctypes.c_uint64, ctypes.c_int64,
            ctypes.c_int32, _dp, _dp, _dp,
        ]
        lib.dtc_energy_sums.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), P(DtcDeviceNoise), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_int32, _dp, _dp, _dp,
        ]
        lib.dtc_prefix_build.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), P(DtcDeviceNoise), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_int32, ctypes.c_int32,
        ]
        lib.dtc_autocorr_prefixed.argtypes = [
            ctypes.c_void_p, P(DtcProblem), P(DtcNoise), P(DtcDeviceNoise), ctypes.c_uint64,
            ctypes.c_int64, ctypes.c_int32, _dp, _dp,
        ]
        lib.dtc_prefix_release.argtypes = [ctypes.c_void_p]
        lib.dtc_plan_groups.argtypes = [ctypes.c_int32, P(ctypes.c_uint64), ctypes.c_int32]
        for name in EXPORTED_SYMBOLS:
            if name not in ("dtc_last_error", "dtc_abi_version"):
                getattr(lib, name).restype = ctypes.c_int
        _lib = lib
        return lib


def check(rc: int) -> None:
    if rc != 0:
        msg = _lib.dtc_last_error().decode() if _lib is not None else "unknown"
        raise DtcError(f"libdtc_hip error {rc}: {msg}")


def as_dptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_dp)


def device_struct(dev) -> "DtcDeviceNoise":
    """dtc_device_noise view of a DeviceNoise (arrays stay owned by ``dev``)."""
    d = DtcDeviceNoise()
    d.p_gate = as_dptr(dev.p_gate)
    d.t1_us = as_dptr(dev.t1_us)
    d.t2_us = as_dptr(dev.t2_us)
    d.gate_ns = float(dev.gate_ns)
    d.anc_factor = float(dev.anc_factor)
    d.readout_p01 = float(dev.readout_p01)
    d.readout_p10 = float(dev.readout_p10)
    return d


def plan_groups(n_bits: int) -> list:
    """Host-only: bit masks of the site groups the engine's passes use."""
    lib = load_library()
    buf = (ctypes.c_uint64 * 16)()
    n = lib.dtc_plan_groups(int(n_bits), buf, 16)
    if n < 0:
        check(n)
    return [int(buf[i]) for i in range(n)]
