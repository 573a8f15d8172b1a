"""Command line mirroring the energy scripts:

    --mode full            autocorr-delta-a-single-qiskit-fast-energy.py (and -energy-envelope)
                           nprobs = [0, 0.001, 0.01, 0.1], accumulated in one noise model
                           (energy.py:209-222); columns energy_p_{nprob}
    --mode ham-comparison  ...-energy-ham-comparison.py: nprobs = [noise_prob];
                           columns energy_{z_only,zz_only,x_only,sum,full}_p_{nprob}
    --mode vs-echo         ...-energy-ham-comparison-vs-echo.py: nprobs = [0.1];
                           columns energy_{with,without}_x_p_{nprob}
    --mode fakebrisbane    ...-energy-fakebrisbane.py: the circuits on the device
                           backend; column energy_p_fakebrisbane = mean over
                           instances of <H>(t), NOT divided by L (as that script
                           saves it); folder energy-data_L{L}-fakebrisbane

Flags as energy.py:26-40; files and folders as the scripts write them
(energy.py:57-61, 229-234; ham-comparison.py:277-280; vs-echo.py:248-251).
Values are ``mean over instances of <H>(t) / L`` except for fakebrisbane.

``--use_fakebackend`` defaults as in each script (1 for vs-echo and fakebrisbane,
0 otherwise).  With 1 the noise is device-like noise from ``--device_calibration``
(FakeBrisbane's own snapshot ships inside qiskit-ibm-runtime and is not available
offline; default: the documented stand-in data/device_standin_L20.json) plus
per-site read-out error, and — as in the scripts — no depolarizing error is added
for the nprob columns.
"""
from __future__ import annotations

import argparse
import os

import numpy as np

from . import energy as en
from .disorder import load_disorder


def build_parser():
    p = argparse.ArgumentParser(description="DTC energy sweep on MI355X (HIP engine)")
    p.add_argument("--mode", choices=("full", "ham-comparison", "vs-echo", "fakebrisbane"),
                   default="full")
    p.add_argument("--L", type=int, default=4)
    p.add_argument("--device_name", type=int, default=0)
    p.add_argument("--inst", type=int, default=1)
    p.add_argument("--randomphi", type=int, default=1)
    p.add_argument("--phi_delta", type=float, default=0.0)
    p.add_argument("--phi_amplitude", type=float, default=1.0)
    p.add_argument("--tf", type=int, default=20)
    p.add_argument("--g", type=float, default=0.97)
    p.add_argument("--noise_prob", type=float, default=0.05)
    p.add_argument("--use_noise", type=int, default=1)
    p.add_argument("--initial_state", type=str, default="vacuum", choices=["vacuum", "neel"])
    p.add_argument("--use_fakebackend", type=int, default=None,
                   help="default: 1 for --mode vs-echo / fakebrisbane, else 0 (as the scripts)")
    p.add_argument("--device_calibration", type=str, default=None,
                   help="calibration JSON for --use_fakebackend 1 (default: the stand-in)")
    p.add_argument("--trajectories", type=int, default=en.ESTIMATOR_SHOTS,
                   help="trajectories per point (default: the estimator's 4096 shots)")
    p.add_argument("--seed", type=int, default=0x5EED0001)
    p.add_argument("--disorder_folder", type=str, default=".")
    p.add_argument("--out_dir", type=str, default=".")
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    L, T = args.L, args.tf
    hs, phis = load_disorder(L, args.inst, args.disorder_folder)
    ts = np.arange(0, T)
    name_args = (args.initial_state, args.g, L, args.inst, args.randomphi, args.phi_delta,
                 args.phi_amplitude, args.noise_prob, args.use_noise)
    use_fake = args.use_fakebackend
    if use_fake is None:
        use_fake = 1 if args.mode in ("vs-echo", "fakebrisbane") else 0
    cal = None
    if use_fake:
        from .cli import DEFAULT_CALIBRATION
        from .device_noise import DeviceCalibration

        cal_path = args.device_calibration or DEFAULT_CALIBRATION
        cal = DeviceCalibration.from_json(cal_path)
        print(f"Device-like noise from {cal_path} ({cal.name})")
    if args.mode == "fakebrisbane":
        e = en.run_energy_device(L, args.g, hs, phis, T, cal, initial_state=args.initial_state,
                                 n_traj=args.trajectories, seed=args.seed)
        cols = {"energy_p_fakebrisbane": e}
        path = os.path.join(args.out_dir, en.energy_folder(L, "fakebrisbane"),
                            en.energy_csv_name("energy_data", *name_args))
    elif args.mode == "full":
        nprobs = [0, 0.001, 0.01, 0.1]
        noisy = bool(args.use_noise)
        res = en.run_energy(L, args.g, hs, phis, T, nprobs, use_noise=int(noisy),
                            initial_state=args.initial_state, n_traj=args.trajectories,
                            seed=args.seed, calibration=cal)
        cols = {f"energy_p_{p}": res[("full", p)] for p in nprobs}
        path = os.path.join(args.out_dir, en.energy_folder(L, "full-ham"),
                            en.energy_csv_name("energy_data", *name_args))
    elif args.mode == "ham-comparison":
        nprobs = [args.noise_prob]
        res = en.run_energy(L, args.g, hs, phis, T, nprobs, use_noise=1,
                            initial_state=args.initial_state, n_traj=args.trajectories,
                            seed=args.seed, calibration=cal,
                            hamiltonian_types=("z_only", "zz_only", "x_only", "full"))
        cols = {}
        for p in nprobs:
            cols[f"energy_z_only_p_{p}"] = res[("z_only", p)]
            cols[f"energy_zz_only_p_{p}"] = res[("zz_only", p)]
            cols[f"energy_x_only_p_{p}"] = res[("x_only", p)]
            cols[f"energy_sum_p_{p}"] = res[("z_only", p)] + res[("zz_only", p)]
            cols[f"energy_full_p_{p}"] = res[("full", p)]
        path = os.path.join(args.out_dir, en.energy_folder(L, "ham-comparison"),
                            en.energy_csv_name("energy_comparison_all", *name_args))
    else:
        nprobs = [0.1]
        res = en.run_energy(L, args.g, hs, phis, T, nprobs, use_noise=1,
                            initial_state=args.initial_state, n_traj=args.trajectories,
                            seed=args.seed, calibration=cal,
                            hamiltonian_types=("full", "z_zz"))
        cols = {}
        for p in nprobs:
            cols[f"energy_with_x_p_{p}"] = res[("full", p)]
            cols[f"energy_without_x_p_{p}"] = res[("z_zz", p)]
        path = os.path.join(args.out_dir, en.energy_folder(L, "ham-comparison"),
                            en.energy_csv_name("energy_comparison", *name_args))
    en.write_energy_csv(path, ts, cols)
    print(f"Energy data saved to {path}")
    if args.mode == "vs-echo":
        p = nprobs[0]
        print(f"saved {write_comprehensive(args, ts, res[('full', p)], res[('z_zz', p)])}")
    return 0


def write_comprehensive(args, ts, e_with, e_without):
    """vs-echo.py:332-448: energies next to the autocorrelator of an existing
    sweep CSV (autocorr_data_L{L}_noiseprob{p}/…_tf{tf}_….csv under --out_dir),
    or the energy-only file when that CSV is absent."""
    import pandas as pd

    L = args.L
    tail = (f"{args.initial_state}_g{args.g}_L{L}_inst{args.inst}_tf{args.tf}"
            f"_randomphi{args.randomphi}_delta{args.phi_delta}_amplitude{args.phi_amplitude}"
            f"_noise{args.noise_prob}_usenoise{args.use_noise}.csv")
    src = os.path.join(args.out_dir, f"autocorr_data_L{L}_noiseprob{args.noise_prob}",
                       "autocorr_data_" + tail)
    data = {"time": ts, "energy_with_x": e_with, "energy_without_x": e_without}
    if os.path.exists(src):
        ac = pd.read_csv(src)
        n = len(ts)

        def fit(v):
            v = np.asarray(v, dtype=float)
            return v[:n] if len(v) >= n else np.concatenate([v, np.full(n - len(v), np.nan)])

        data["autocorr_forward"] = fit(ac["av_autocorr"].values)
        data["autocorr_echo"] = fit(ac["av_autocorr_echo"].values)
        data["minus_autocorr_echo"] = -fit(ac["av_autocorr_echo"].values)
        name = "comprehensive_data_" + tail
    else:
        name = "comprehensive_data_energy_only_" + tail
    path = os.path.join(args.out_dir, en.energy_folder(L, "ham-comparison"), name)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    pd.DataFrame(data).to_csv(path, index=False)
    return path
