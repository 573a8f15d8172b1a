import importlib, os, sys, time
import numpy as np
sys.path.insert(0, "/root/repo")
pkg = importlib.import_module("noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd")
import bench
hs, phis = bench.load_disorder_row(20)
eng = pkg.DtcEngine(0)
for B in (4, 8, 16, 64, 256):
    spec = pkg.SweepSpec(L=20, T=60, hs=hs, phis=phis, g=0.97, noise_prob=0.05)
    eng.autocorr(spec, B, batch=B, want_echo=False)
    eng.reset_stats(); eng.set_profiling(True)
    eng.autocorr(spec, B, batch=B, want_echo=False, traj_offset=99)
    eng.set_profiling(False)
    st = eng.kernel_stats()[0]
    us = st["total_ms"] / st["launches"] * 1e3
    print(f"fwd-only B={B}: kdk {us:.1f} us  {32*2**20*B/us/1e3:.0f} GB/s  ({st['launches']} launches)", flush=True)
