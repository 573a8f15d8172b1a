"""Development probe (not the product): can a cache-resident C2 schedule beat the
HBM-batched one at HEAD?  Runs the C2 sweep (L=20, T=30, p=0.05, hs/phis_L20 row 0)
as E engines x batch b (each engine its own HIP stream, driven from its own host
thread, so E batches of b states are in flight at once: F + E footprint
E * b * 32 MiB) and prints the aggregate throughput and, per config, the engines'
launch-weighted K-D-K kernel time (HIP events on each engine stream) as GB/s of
algorithmic bytes (32 B per amplitude per launch, 48 for the dual passes).
usage (GPU box): python tools/resident_sweep.py [--ntraj N] 1x1024 1x16 1x8 2x4 4x2 4x1"""
import argparse
import importlib
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402,F401  (one HIP runtime per process, see _capi)

pkg = importlib.import_module(
    "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd")
import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ntraj", type=int, default=256, help="trajectories per config (all engines)")
ap.add_argument("configs", nargs="+")
a = ap.parse_args()

hs, phis = bench.load_disorder_row(20)
spec = pkg.SweepSpec(L=20, T=30, hs=hs, phis=phis, g=0.97, noise_prob=0.05)
LO = 0  # DTC_KERNEL_LO_PASS: every pass that applies the diagonal and stores

for cfg in a.configs:
    ne, b = (int(x) for x in cfg.split("x"))
    per_eng = max(b, a.ntraj // ne)
    engs = [pkg.DtcEngine(0) for _ in range(ne)]
    for e in engs:  # warm: buffers, tables, code objects
        e.autocorr(spec, min(per_eng, 2 * b), batch=b)
    for e in engs:
        e.reset_stats()
        e.set_profiling(True)

    def run(k):
        engs[k].autocorr(spec, per_eng, batch=b, traj_offset=10000 + k * per_eng)

    th = [threading.Thread(target=run, args=(k,)) for k in range(ne)]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    el = time.perf_counter() - t0
    n = 0
    ms = 0.0
    by = 0.0
    kern = 0.0
    for e in engs:
        st = e.kernel_stats()
        n += st[LO]["launches"]
        ms += st[LO]["total_ms"]
        by += st[LO]["bytes"]
        kern += sum(v["total_ms"] for v in st.values())
        e.set_profiling(False)
        e.close()
    rate = 464 * per_eng * ne / el
    print(f"{ne} x batch {b:5d} (footprint {ne * b * 32} MiB): {rate:9.0f} periods*inst/s  "
          f"wall {el:.3f} s  kdk {ms / max(n, 1) * 1e3:8.1f} us/launch  "
          f"{by / (ms / 1e3) / 1e9 if ms else 0:6.0f} GB/s per stream  "
          f"sum kernel time / wall {kern / 1e3 / el:.2f}", flush=True)
