"""The C-ABI library loads without a GPU and exports every function that
include/dtc.h declares; error paths work without touching a device."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, "include", "dtc.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|int32_t|const char\*)\s+(dtc_\w+)\s*\(", src,
                                 re.M)))


def test_header_declares_python_binding_table(pkg):
    assert _declared() == sorted(pkg._capi.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol(pkg):
    lib = ctypes.CDLL(pkg._capi.LIB_PATH)
    for name in _declared():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", pkg._capi.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dtc_\w+)", out))
    assert set(_declared()) <= exported


def test_library_is_gfx950_code_object(pkg):
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readobj", "--sections",
                          pkg._capi.LIB_PATH], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(pkg._capi.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"dtc_kdk_pass" in blob and b"dtc_kick_pass" in blob


def test_abi_version_and_null_errors(pkg):
    lib = pkg._capi.load_library()
    assert lib.dtc_abi_version() == 12 == pkg._capi.ABI_VERSION
    # null context / arguments are rejected before any device call
    assert lib.dtc_autocorr(None, None, None, 0, 0, 1, None, None, None) == -1
    assert b"null" in lib.dtc_last_error()
    assert lib.dtc_close(None) == 0
    assert lib.dtc_set_profiling(None, 1) == -1
    assert lib.dtc_lightcone_counts(None, None) == -1
    assert lib.dtc_schedule_counts(None, None) == -1
    assert lib.dtc_shard_kick_exchange_slice(None, None, None, None, 0, 0, 1, 0, 0, 0, None) == -1


def test_open_without_gpu_fails_loudly(pkg):
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(pkg._capi.DtcError):
        pkg.DtcEngine(0)


def test_missing_library_raises(pkg, monkeypatch, tmp_path):
    monkeypatch.setattr(pkg._capi, "_lib", None)
    with pytest.raises(pkg._capi.DtcError, match="not built"):
        pkg._capi.load_library(str(tmp_path / "nope.so"))
