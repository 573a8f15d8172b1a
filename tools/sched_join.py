"""Development: join a DTC_PRINT_SCHED schedule dump with its rocprofv3 kernel
trace (tools/sched_trace.sh) and print per-role launch durations.
Usage: python tools/sched_join.py gpurun_out/st_<tag> [...]"""
import collections
import sys

import pandas as pd

for base in sys.argv[1:]:
    sched = [l.split() for l in open(base + ".sched") if l.startswith("sched ")]
    k = pd.read_csv(base + "/kt_kernel_trace.csv").sort_values("Dispatch_Id")
    k = k[~k.Kernel_Name.str.contains("prep|reduce|rocclr|dbg_")]
    assert len(k) % len(sched) == 0, (len(k), len(sched))
    names = k.Kernel_Name.str.replace(r"\(.*", "", regex=True).str.replace("void dtc::", "")
    dur = ((k.End_Timestamp - k.Start_Timestamp) / 1e6).tolist()
    stats = collections.defaultdict(list)
    for i, (n, d) in enumerate(zip(names, dur)):
        f = sched[i % len(sched)]
        stats[(n, f[2], f[3], f[8], f[9])].append(d)
    for key, v in sorted(stats.items()):
        print(base.split("/")[-1], *key, len(v), f"{sum(v) / len(v):.3f} [{min(v):.3f}, {max(v):.3f}]")
