"""Command line mirroring autocorr-delta-a-single-qiskit-fast-controlled-g.py
(``--script controlled-g``, defaults of controlled-g.py:93-110) and
-g-optimization.py (``--script g-optimization``, defaults of gopt.py:91-111):
realtime adaptive run, then fixed-g comparisons at g_initial and 0.97, written
to controlled-autocorr_data_L{L}/ with the scripts' file names and columns."""
from __future__ import annotations

import argparse

import numpy as np

from . import control as ct
from .disorder import load_disorder

DEFAULTS = {
    "controlled-g": {"L": 4, "inst": 10, "use_optimization": 0},
    "g-optimization": {"L": 20, "inst": 1, "use_optimization": 1},
}


def build_parser(script="controlled-g"):
    d = DEFAULTS[script]
    p = argparse.ArgumentParser(description=f"adaptive-g DTC sweep ({script}) on MI355X")
    p.add_argument("--script", choices=tuple(DEFAULTS), default=script)
    p.add_argument("--L", type=int, default=d["L"])
    p.add_argument("--device_name", type=int, default=0)
    p.add_argument("--inst", type=int, default=d["inst"])
    p.add_argument("--randomphi", type=int, default=1)
    p.add_argument("--phi_delta", type=float, default=0.0)
    p.add_argument("--phi_amplitude", type=float, default=1.0)
    p.add_argument("--tf", type=int, default=20)
    p.add_argument("--g", type=float, default=0.84)
    p.add_argument("--noise_prob", type=float, default=0.05)
    p.add_argument("--use_noise", type=int, default=1)
    p.add_argument("--initial_state", type=str, default="vacuum", choices=["vacuum", "neel"])
    p.add_argument("--use_fakebackend", type=int, default=0,
                   help="1: device-like noise from --device_calibration (FakeBrisbane's own "
                        "calibration is not available offline)")
    p.add_argument("--device_calibration", type=str, default=None,
                   help="calibration JSON for --use_fakebackend 1 (default: the stand-in)")
    p.add_argument("--target_echo", type=float, default=1.0)
    p.add_argument("--feedback_gain", type=float, default=0.01)
    p.add_argument("--exponential_feedback", type=int, default=1)
    p.add_argument("--decay_compensation", type=float, default=0.1)
    p.add_argument("--g_min", type=float, default=0.84)
    p.add_argument("--g_max", type=float, default=1.0)
    p.add_argument("--use_optimization", type=int, default=d["use_optimization"])
    p.add_argument("--optimization_iterations", type=int, default=5)
    p.add_argument("--prefix_cache", type=int, default=1,
                   help="optimisation: evaluate candidates from the shared t-period forward "
                        "states (0: a full t+1-period run per evaluation, as the reference)")
    p.add_argument("--shots", type=int, default=1024)
    p.add_argument("--seed", type=int, default=0x5EED0001)
    p.add_argument("--disorder_folder", type=str, default=".")
    p.add_argument("--out_dir", type=str, default=".")
    return p


def main(argv=None):
    pre = argparse.ArgumentParser(add_help=False)
    pre.add_argument("--script", choices=tuple(DEFAULTS), default="controlled-g")
    known, _ = pre.parse_known_args(argv)
    args = build_parser(known.script).parse_args(argv)
    if args.script == "controlled-g" and args.use_optimization:
        raise SystemExit("--use_optimization belongs to --script g-optimization")
    cfg = ct.ControllerConfig(args.target_echo, args.feedback_gain, args.exponential_feedback,
                              args.decay_compensation, args.g_min, args.g_max,
                              args.use_optimization, args.optimization_iterations,
                              args.prefix_cache)
    L, T = args.L, args.tf
    hs, phis = load_disorder(L, args.inst, args.disorder_folder)
    device = None
    if args.use_fakebackend:
        # ctrlg.py:246-250 runs on FakeBrisbane(); its calibration is not
        # available offline: device-like noise from a calibration file
        from .cli import DEFAULT_CALIBRATION
        from .device_noise import DeviceCalibration

        cal_path = args.device_calibration or DEFAULT_CALIBRATION
        cal = DeviceCalibration.from_json(cal_path)
        print(f"Device-like noise from {cal_path} ({cal.name})")
        device = cal.device_noise(L)
    common = dict(noise_prob=args.noise_prob, use_noise=args.use_noise,
                  initial_state=args.initial_state, shots=args.shots, device=device)
    ad = ct.realtime_adaptive(L, T, hs, phis, args.g, cfg, seed=args.seed, log=print, **common)
    std84 = ct.fixed_g_sweep(L, T, hs, phis, args.g, seed=args.seed + 1, **common)
    std97 = ct.fixed_g_sweep(L, T, hs, phis, 0.97, seed=args.seed + 2, **common)
    paths = ct.write_controlled_outputs(
        args.out_dir, args.initial_state, L, args.inst, args.g, cfg, ad, std84, std97,
        (args.randomphi, args.phi_delta, args.phi_amplitude, args.noise_prob, args.use_noise),
        optimization_script=args.script == "g-optimization")
    for p in paths:
        print(f"saved {p}")
    print(f"average g {np.mean(ad.g):.4f}, final echo {np.mean(ad.echo[:, -1]):.4f}")
    return 0
