"""Summarise a rocprofv3 FETCH_SIZE / WRITE_SIZE pair of passes into the
per-launch HBM byte counts bench.py reports as roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes
of 16-B-per-lane coalesced streaming reads -> x2; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Units: KiB.
usage: python tools/pmc_summary.py <prof_dir> <out.json> <batch> <L>
"""
import json
import sys

import pandas as pd


def main(prof, out, batch, L):
    fe = pd.read_csv(f"{prof}/fetch_counter_collection.csv")
    wr = pd.read_csv(f"{prof}/write_counter_collection.csv")
    res = {"source": prof, "batch": batch, "L": L,
           "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB), gfx950 FETCH_SIZE halving"}
    alg = 32.0 * (1 << max(L, 12)) * batch
    for kname, key in (("dtc_kdk_pass", "lo_pass"), ("dtc_kick_pass", "hi_pass")):
        f = fe[fe.Kernel_Name.str.contains(kname)]["Counter_Value"].mean() * 1024
        w = wr[wr.Kernel_Name.str.contains(kname)]["Counter_Value"].mean() * 1024
        res[key] = {"kernel": kname, "fetch_bytes_raw": f, "write_bytes": w,
                    "hbm_bytes_per_launch": 2 * f + w,
                    "algorithmic_bytes_per_launch": alg,
                    "ratio_to_algorithmic": (2 * f + w) / alg}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]))
