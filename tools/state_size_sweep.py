"""Development measurement (not the product): pass-kernel HBM rate vs state
size at a fixed 16 GiB per launch.  Forward-only noiseless sweeps (probe
measured every period) of B states of L sites, B * 2^L = 2^30 amplitudes, so
every launch moves the same 32 GiB; prints the engine's HIP-event rates of the
K-D-K passes (diagonal) and the kick-only passes.  Usage (GPU box):
    python tools/state_size_sweep.py [L ...]"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module(
    "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd")


def run(L, T=12):
    B = (1 << 30) >> L
    rng = np.random.default_rng(L)
    hs = rng.uniform(0, 2 * np.pi, (1, L))
    phis = rng.uniform(-np.pi, np.pi, (1, L - 1))
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.97, use_noise=0)
    eng = pkg.DtcEngine(0)
    eng.autocorr(spec, B, want_echo=False, batch=B)  # warm-up
    eng.reset_stats()
    eng.set_profiling(True)
    eng.autocorr(spec, B, want_echo=False, batch=B)
    eng.set_profiling(False)
    st = eng.kernel_stats()
    out = []
    for k, name in ((0, "kdk"), (1, "kick")):
        s = st[k]
        if s["launches"]:
            out.append(f"{name} {s['launches']:3d} x {s['total_ms'] / s['launches']:7.3f} ms "
                       f"{s['bytes'] / (s['total_ms'] / 1e3) / 1e9:7.0f} GB/s")
    print(f"L={L:2d} B={B:5d}  " + "   ".join(out), flush=True)
    eng.close()


if __name__ == "__main__":
    for L in [int(a) for a in sys.argv[1:]] or [20, 22, 24, 26, 28]:
        run(L)
