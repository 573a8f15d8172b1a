"""Development probe (not the product): one C2-shaped sweep (L=20, T=30,
hs/phis_L20 row 0, B=1024) with a chosen noise probability and polarization,
for kernel traces of the pass kernels under other kick statistics.
usage (GPU box): python tools/c2_variant.py [--noise p] [--pol x|y] [--echo 0|1]"""
import argparse
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process, see _capi)

pkg = importlib.import_module(
    "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd")
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--noise", type=float, default=0.05)
ap.add_argument("--pol", default="x")
ap.add_argument("--g", type=float, default=0.97)
a = ap.parse_args()
hs, phis = bench.load_disorder_row(20)
spec = pkg.SweepSpec(L=20, T=30, hs=hs, phis=phis, g=a.g, noise_prob=a.noise,
                     use_noise=1 if a.noise else 0, polarization=a.pol)
with pkg.DtcEngine(0) as eng:
    out = eng.autocorr(spec, 1024, seed=0x5EED0001, batch=1024)
    print("echo t0..3", out["echo"][0, :, :4].mean(axis=0))
