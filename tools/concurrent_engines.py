"""Development probe (not the product): does running two C2 sweeps at once on
one GPU (two engines, two HIP streams, out of phase) beat one sweep of the
same total batch?  If so, overlapping the VALU-bound light-cone passes with
the HBM-bound K-D-K passes of another chain pays.
usage (GPU box): python tools/concurrent_engines.py [total_traj] [reps]"""
import importlib
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

pkg = importlib.import_module(
    "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd")
import bench  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
hs, phis = bench.load_disorder_row(20)
spec = pkg.SweepSpec(L=20, T=30, hs=hs, phis=phis, g=0.97, noise_prob=0.05)
torch.cuda.set_device(0)
e1, e2 = pkg.DtcEngine(0), pkg.DtcEngine(0)
unit = N * 464
e1.autocorr(spec, N, batch=N)
e2.autocorr(spec, N // 2, batch=N // 2)
e1.autocorr(spec, N // 2, batch=N // 2)
torch.cuda.synchronize()
t0 = time.time()
for r in range(reps):
    e1.autocorr(spec, N, batch=N, traj_offset=r * N)
torch.cuda.synchronize()
one = unit * reps / (time.time() - t0)
print(f"one engine, {N} per call: {one:.0f} periods*traj/s", flush=True)


durs = {0: [], 1: []}


def run(k, eng, off, delay):
    time.sleep(delay)
    for r in range(reps):
        t = time.time()
        eng.autocorr(spec, N // 2, batch=N // 2, traj_offset=off + r * N)
        durs[k].append(time.time() - t)


half_step = N * 464 / one / 2  # seconds: half of one N-trajectory call
t0 = time.time()
th = [threading.Thread(target=run, args=(k, e, o, d))
      for k, e, o, d in ((0, e1, 0, 0.0), (1, e2, N // 2, half_step / 2))]
for t in th:
    t.start()
for t in th:
    t.join()
torch.cuda.synchronize()
two = unit * reps / (time.time() - t0)
print(f"two engines concurrently, {N // 2} each, second started {half_step / 2:.2f} s late: "
      f"{two:.0f} periods*traj/s ({two / one:.3f}x)", flush=True)
import numpy as np  # noqa: E402
mid = [d for k in (0, 1) for d in durs[k][1:-1]]
print(f"  call durations (s): {[round(d, 3) for d in durs[0]]} / {[round(d, 3) for d in durs[1]]}; "
      f"middle calls median {np.median(mid):.3f} s = {(N // 2) * 464 * 2 / np.median(mid):.0f} "
      f"periods*traj/s for the pair", flush=True)
t0 = time.time()
for r in range(reps):
    e1.autocorr(spec, N // 2, batch=N // 2, traj_offset=r * N)
    e1.autocorr(spec, N // 2, batch=N // 2, traj_offset=r * N + N // 2)
torch.cuda.synchronize()
seq = unit * reps / (time.time() - t0)
print(f"one engine, two calls of {N // 2}: {seq:.0f} periods*traj/s", flush=True)
e1.close()
e2.close()
