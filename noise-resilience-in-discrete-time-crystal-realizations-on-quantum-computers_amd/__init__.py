"""MI355X-native simulator for the DTC autocorrelator sweep.

Reference path: autocorr-delta-a-single-qiskit-fast*.py.
The compute path is the gfx950 HIP library ``lib/libdtc_hip.so`` behind the
C ABI in ``include/dtc.h``; this package is the host-side mirror of the
reference's interface (AerSimulator-shaped facade, sweep drivers, CSV
writer).

The directory name is not a Python identifier; import it with
``importlib.import_module(PACKAGE_NAME)`` after putting the repo root on
``sys.path`` (``__graft_entry__.load_package()`` does that).
"""
from __future__ import annotations

PACKAGE_NAME = "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd"

from . import _capi  # noqa: E402
from .kicks import kick_table, POLARIZATIONS, rx, ry  # noqa: E402
from .disorder import load_disorder, generate_disorder, save_disorder_to_csv  # noqa: E402
from .engine import DtcEngine, SweepSpec, energy_init_mask, init_mask, N_ANCILLA_NOISY_GATES  # noqa: E402
from . import circuit, aer, sweep, distributed, sharded, energy, envelopes, control  # noqa: E402
from . import cli, energy_cli, control_cli  # noqa: E402
from .circuit import QuantumCircuit, transpile_aer_basis  # noqa: E402
from .aer import AerSimulator, DtcSimulator, NoiseModel, depolarizing_error  # noqa: E402
from .device_noise import DeviceNoise, DeviceCalibration  # noqa: E402
from . import device_noise  # noqa: E402
from .sweep import (run_sweep, get_instances, get_single_out,  # noqa: E402
                    compute_z_expectation, write_autocorr_csv)

__all__ = [
    "PACKAGE_NAME", "DtcEngine", "SweepSpec", "kick_table", "POLARIZATIONS", "rx", "ry",
    "load_disorder", "generate_disorder", "save_disorder_to_csv", "init_mask", "energy_init_mask",
    "N_ANCILLA_NOISY_GATES", "QuantumCircuit", "transpile_aer_basis", "AerSimulator",
    "DtcSimulator", "NoiseModel", "depolarizing_error", "run_sweep", "get_instances",
    "get_single_out", "compute_z_expectation", "write_autocorr_csv", "circuit", "aer",
    "sweep", "distributed", "sharded", "energy", "envelopes", "control", "cli", "energy_cli",
    "control_cli", "DeviceNoise", "DeviceCalibration", "device_noise",
]
