"""Command line mirroring autocorr-delta-a-single-qiskit-fast.py (and the
-polarization / -circular-polarization / -xy-cycle / -shots variants).

    python dtc_autocorr.py --L 20 --tf 30 --g 0.97 --noise_prob 0.05

Flags are those of fast.py:25-37 (+ --polarization / --circular_frequency of
...-circular-polarization.py:42-43, --shots of ...-shots.py) plus engine
options.  Output: the same folder and ``autocorr_data_*.csv`` as fast.py:56-59,
259-270 (and optionally the gate_counts CSVs of fast.py:193-197), so the
reference's draw-*.py scripts read it unchanged.  ``--device_name`` and
``--randomphi/--phi_delta/--phi_amplitude`` only enter file names, as in the
reference.  Under torchrun the trajectories are sharded over ranks (one GPU
per rank) and gathered on rank 0.
"""
from __future__ import annotations

import argparse
import os
import time

import numpy as np

from .device_noise import DeviceCalibration
from .disorder import load_disorder
from .engine import SweepSpec
from .kicks import POLARIZATIONS
from . import sweep as sw

# documented stand-in calibration (data/device_standin_L20.json): the reference's
# FakeBrisbane snapshot is not available offline
DEFAULT_CALIBRATION = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                   "data", "device_standin_L20.json")


def build_parser():
    p = argparse.ArgumentParser(description="DTC autocorrelator sweep on MI355X (HIP engine)")
    p.add_argument("--L", type=int, default=4, help="Number of qubits")
    p.add_argument("--device_name", type=int, default=0, help="Device name (unused, as in fast.py)")
    p.add_argument("--inst", type=int, default=1, help="Number of disorder instances")
    p.add_argument("--randomphi", type=int, default=1, help="Prethermal=0 or DTC=1 (file name)")
    p.add_argument("--phi_delta", type=float, default=0.0, help="Phi delta parameter (file name)")
    p.add_argument("--phi_amplitude", type=float, default=1.0, help="Phi amplitude (file name)")
    p.add_argument("--tf", type=int, default=50, help="end time")
    p.add_argument("--g", type=float, default=0.97, help="kick strength g (RX(pi g))")
    p.add_argument("--noise_prob", type=float, default=0.05, help="depolarizing probability")
    p.add_argument("--use_noise", type=int, default=1, help="0=no noise, 1=apply noise")
    p.add_argument("--initial_state", type=str, default="vacuum", choices=["vacuum", "neel"])
    p.add_argument("--use_fakebackend", type=int, default=0,
                   help="1 = device-like noise (thermal relaxation + depolarizing + read-out) "
                        "from --device_calibration; FakeBrisbane's own data is not available "
                        "offline")
    p.add_argument("--device_calibration", type=str, default=DEFAULT_CALIBRATION,
                   help="calibration JSON for --use_fakebackend 1 (device-like noise)")
    p.add_argument("--polarization", type=str, default="x", choices=list(POLARIZATIONS))
    p.add_argument("--circular_frequency", type=float, default=1.0)
    # engine options
    p.add_argument("--shots", type=int, default=1024,
                   help="emulate the reference's shot estimator (0 = trajectory mean)")
    p.add_argument("--trajectories", type=int, default=0,
                   help="noisy trajectories per instance (default = shots)")
    p.add_argument("--seed", type=int, default=0x5EED0001)
    p.add_argument("--disorder_folder", type=str, default=".")
    p.add_argument("--out_dir", type=str, default=".")
    p.add_argument("--t_offset", type=int, default=0,
                   help="periods at time t = t + t_offset (1 for the controlled-g scripts)")
    p.add_argument("--gate_counts", type=int, default=0, help="also write gate_counts_*.csv")
    p.add_argument("--batch", type=int, default=0, help="states per device batch (0 = auto)")
    p.add_argument("--independent_t", type=int, default=0,
                   help="1 = every t from its own trajectories (uncorrelated across t, as the "
                        "reference's circuit per t, fast.py:219-221; O(T^2) periods); 0 = the "
                        "echo branches off one forward trajectory (correlated across t)")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    L, T = args.L, args.tf
    device = None
    if args.use_fakebackend:
        # fast.py:77-79 uses FakeBrisbane's calibration (not available offline):
        # a user-supplied calibration file drives the device-like noise path
        cal = DeviceCalibration.from_json(args.device_calibration)
        device = cal.device_noise(L)
        print(f"Device-like noise from {args.device_calibration} ({cal.name})")
    hs, phis = load_disorder(L, args.inst, args.disorder_folder)
    spec = SweepSpec(L=L, T=T, hs=hs, phis=phis, g=args.g, polarization=args.polarization,
                     circular_frequency=args.circular_frequency,
                     initial_state=args.initial_state, noise_prob=args.noise_prob,
                     use_noise=args.use_noise, t_offset=args.t_offset, device=device)
    shots = args.shots or None
    if spec.p == 0 and device is None:
        n_traj = 1
    else:
        n_traj = args.trajectories or (shots or 1024)
    if shots and spec.p > 0 and device is None and n_traj != shots:
        raise SystemExit("--trajectories must equal --shots when emulating shots (use --shots 0 "
                         "for trajectory means)")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    t0 = time.time()
    if world > 1:
        from .distributed import sharded_sweep

        res = sharded_sweep(spec, n_traj, shots=shots, seed=args.seed, batch=args.batch,
                            independent_t=bool(args.independent_t))
        if rank != 0:
            return 0
    else:
        res = sw.run_sweep(spec, n_traj=n_traj, shots=shots, seed=args.seed, batch=args.batch,
                           independent_t=bool(args.independent_t))
    elapsed = time.time() - t0
    print(f"Completed forward+echo sweep in {elapsed:.2f}s "
          f"({spec.n_inst} instance(s) x {n_traj} trajectories x {T} times)")

    folder = os.path.join(args.out_dir, sw.folder_name(L, args.noise_prob, args.use_fakebackend))
    name = sw.autocorr_csv_name(args.initial_state, args.g, L, args.inst, args.tf, args.randomphi,
                                args.phi_delta, args.phi_amplitude, args.noise_prob,
                                args.use_noise)
    path = sw.write_autocorr_csv(os.path.join(folder, name), np.arange(0, T),
                                 res.av_autocorr, res.av_autocorr_echo)
    print(f"Autocorrelation data saved to {path}")
    if args.gate_counts:
        sw.write_gate_counts(folder, spec, args.polarization, args.g,
                             circular_frequency=args.circular_frequency)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
