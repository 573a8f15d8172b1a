"""Test configuration.

`-m "not gpu"` tests run in the build container (no GPU): the oracles, host
logic, fixtures and the C-ABI symbol table.  `-m gpu` tests call the HIP
engine through the C ABI on an MI355X and compare with the oracle.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def _ensure_built():
    lib = os.path.join(ROOT, "oracle", "liboracle.so")
    hip = os.path.join(ROOT, "noise-resilience-in-discrete-time-crystal-realizations-on-"
                       "quantum-computers_amd", "lib", "libdtc_hip.so")
    if not (os.path.exists(lib) and os.path.exists(hip)):
        subprocess.run(["make", "-C", ROOT, "-j", "4"], check=True,
                       stdout=subprocess.DEVNULL)


_ensure_built()


@pytest.fixture(scope="session")
def pkg():
    from __graft_entry__ import load_package

    return load_package()


@pytest.fixture(scope="session")
def golden():
    import json

    out = {}
    for name in ("disorder", "aer_autocorr", "gate_counts"):
        with open(os.path.join(GOLDEN, name + ".json")) as f:
            out[name] = json.load(f)
    return out


@pytest.fixture(scope="session")
def engine(pkg):
    eng = pkg.DtcEngine(0)
    yield eng
    eng.close()
