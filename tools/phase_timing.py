"""Development tool: per-workgroup phase timing of the K-D-K pass.

Build the instrumented library first (SHAPE = 3 records K-D-K passes):
  hipcc --offload-arch=gfx950 -O3 -fPIC -shared -std=c++17 -DDTC_PHASE_TIMING=3 \\
      <pkg>/csrc/dtc_kernels.hip <pkg>/csrc/dtc_engine.cpp -o build/libdtc_timing.so
then: DTC_LIB=build/libdtc_timing.so python tools/phase_timing.py [batch] [T] [probe|energy|zsite]
Each workgroup's wave 0 stores s_memtime at: start, setup loads landed, tables
ready (barrier), pre-kick rounds done, diagonal done, post-kick rounds done,
stores issued.  The buffer keeps the last recorded launch."""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

pkg = importlib.import_module(
    "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd")
import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
T = int(sys.argv[2]) if len(sys.argv) > 2 else 4
hs, phis = bench.load_disorder_row(20)
spec = pkg.SweepSpec(L=20, T=T, hs=hs, phis=phis, g=0.97, noise_prob=0.05)
torch.cuda.set_device(0)
n_tiles = 256
buf = torch.zeros(B * n_tiles * 8, dtype=torch.int64, device="cuda")
os.environ["DTC_DBG_PTR"] = str(buf.data_ptr())
eng = pkg.DtcEngine(0)
if len(sys.argv) > 3 and sys.argv[3] == "energy":
    eng.energy(spec, B, batch=B)
elif len(sys.argv) > 3 and sys.argv[3] == "zsite":
    eng.autocorr(spec, B, batch=B, want_zsite=True, want_echo=False)
else:
    eng.autocorr(spec, B, batch=B)
torch.cuda.synchronize()
a = buf.cpu().numpy().reshape(-1, 8).astype(np.uint64)
nibs = (a[:, 0] >> np.uint64(60)).astype(int)
a = (a & np.uint64((1 << 60) - 1)).astype(np.int64)
for nb in sorted(set(nibs.tolist())):
    sel = a[nibs == nb]
    if nb == 0 or len(sel) == 0:
        continue
    rt0 = sel[:, 7] & 0xffffffff
    rtd = (sel[:, 7] >> 32) & ((1 << 28) - 1)
    span = (rt0 + rtd).max() - rt0.min()   # 10 ns ticks
    life = sel[:, 6] - sel[:, 0]
    print(f"NIBS={nb}: {len(sel)} workgroups, launch span {span * 10 / 1000:.1f} us, "
          f"median lifetime {np.median(life):.0f} clk = {np.median(rtd) * 10 / 1000:.2f} us, "
          f"mean concurrency {rtd.sum() / span:.0f} workgroups")
    d = np.diff(sel[:, :7], axis=1)
    life = sel[:, 6] - sel[:, 0]
    names = ["issue+setup-loads", "setup(barrier)", "pre-rounds", "diag", "post-rounds", "store"]
    for i, n in enumerate(names):
        print(f"   {n:20s} median {np.median(d[:, i]):8.0f}  mean {d[:, i].mean():8.0f}  "
              f"p90 {np.percentile(d[:, i], 90):8.0f}")
