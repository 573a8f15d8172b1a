"""Development probe (GPU box): the schedule and K-D-K byte accounting of one
autocorr call with and without the dual forward+echo-start pass.  Needs a
development library (engine built with -DDTC_DEV_KNOBS, e.g. devlib/dev.so):
DTC_PRINT_SCHED=1 makes it list every launch on stderr.
usage: DTC_LIB=devlib/dev.so python tools/dual_sched_probe.py L T pol state toff p [no_dual]
"""
import importlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
from helpers import random_disorder  # noqa: E402

PKG = "noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd"


def main():
    L, T = int(sys.argv[1]), int(sys.argv[2])
    pol, state, toff, p = sys.argv[3], sys.argv[4], int(sys.argv[5]), float(sys.argv[6])
    if len(sys.argv) > 7 and sys.argv[7] == "no_dual":
        os.environ["DTC_NO_DUAL"] = "1"
    os.environ["DTC_PRINT_SCHED"] = "1"
    pkg = importlib.import_module(PKG)
    rng = np.random.default_rng(L * 5 + T)
    hs, phis = random_disorder(rng, L, 2)
    spec = pkg.SweepSpec(L=L, T=T, hs=hs, phis=phis, g=0.93, noise_prob=p, polarization=pol,
                         initial_state=state, t_offset=toff)
    with pkg.DtcEngine(0) as eng:
        eng.set_profiling(True)
        eng.autocorr(spec, 3, seed=19)
        st = eng.kernel_stats()
    amps = 3 * (1 << max(L, 12))
    for k, name in pkg._capi.KERNEL_NAMES.items():
        s = st[k]
        if s["launches"]:
            print(f"kind {k} launches {s['launches']} bytes/amp {s['bytes'] / amps:.1f}", flush=True)


if __name__ == "__main__":
    main()
