#!/usr/bin/env python3
"""Write the disorder inputs of the large configs, which
the reference does not ship: generate_disorder.py:16-20 semantics (A=1, delta=0,
randomphi=1) with a fixed seed, in its CSV format (headers h_i / phi_i).

    python tools/make_large_disorder.py   # -> data/hs_L28.csv, phis_L28.csv, hs_L34.csv, phis_L34.csv
"""
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
pkg = importlib.import_module(
    "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd")

CONFIGS = {28: (256, 28), 34: (8, 34)}  # L: (instances, seed)

if __name__ == "__main__":
    out = os.path.join(ROOT, "data")
    for L, (inst, seed) in CONFIGS.items():
        pkg.disorder.save_disorder_to_csv(L, inst, folder=out, seed=seed,
                                          hs_name=f"hs_L{L}.csv", phis_name=f"phis_L{L}.csv")
        print(f"L={L}: {inst} instances (seed {seed}) -> {out}")
