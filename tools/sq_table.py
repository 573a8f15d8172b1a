"""Per-kernel, per-wave means of rocprofv3 --pmc SQ counter passes (the
p*_counter_collection.csv files tools/pmc_sq.sh writes) as a markdown table.
SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles
(MI355X_MICROARCH.md §PMC); every counter is divided by SQ_WAVES of the same
kernel (from the first pass).
usage: python tools/sq_table.py <prof_dir> [kernel substring ...]"""
import glob
import sys

import pandas as pd


def main(prof, pats):
    frames = [pd.read_csv(f) for f in sorted(glob.glob(f"{prof}/p*_counter_collection.csv"))]
    df = pd.concat(frames)
    df["k"] = df.Kernel_Name.str.replace(r"\(dtc::PassArgs\)", "", regex=True).str.replace(
        "void dtc::", "", regex=False)
    if pats:
        df = df[df.k.apply(lambda s: any(p in s for p in pats))]
    tab = df.groupby(["k", "Counter_Name"]).Counter_Value.mean().unstack()
    waves = tab["SQ_WAVES"]
    cols = [c for c in ["SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                        "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                        "SQ_WAIT_INST_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_ACTIVE_INST_LDS",
                        "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_BUSY_CYCLES"] if c in tab]
    print("| kernel | waves/launch | " + " | ".join(c.replace("SQ_", "") for c in cols) + " |")
    print("|---|---|" + "---|" * len(cols))
    for k, row in tab.iterrows():
        w = row["SQ_WAVES"]
        vals = [row[c] / w if c != "SQ_BUSY_CYCLES" else row[c] for c in cols]
        print(f"| {k} | {w:.0f} | " + " | ".join(f"{v:.0f}" for v in vals) + " |")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
