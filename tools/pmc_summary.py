"""Summarise a rocprofv3 FETCH_SIZE / WRITE_SIZE pair of passes into the
per-launch HBM byte counts bench.py reports as roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE counts half the bytes
of 16-B-per-lane coalesced streaming reads -> x2; WRITE_SIZE is exact for
16-B-per-lane streaming stores.  Units: KiB.  Algorithmic bytes per launch:
32 B per amplitude for a pass that reads and stores its states, 16 B for one
that only stores (the basis-synthesising first pass: no fetch) or only reads
(the measure-only light-cone / final passes).
usage: python tools/pmc_summary.py <prof_dir> <out.json> <batch> <L> [bench args]
"""
import json
import sys

import pandas as pd


def main(prof, out, batch, L, bench_args=""):
    fe = pd.read_csv(f"{prof}/fetch_counter_collection.csv")
    wr = pd.read_csv(f"{prof}/write_counter_collection.csv")
    res = {"source": prof, "batch": batch, "L": L, "bench_args": bench_args,
           "correction": "hbm = 2*FETCH_SIZE + WRITE_SIZE (KiB), gfx950 FETCH_SIZE halving"}
    amps = float(1 << max(L, 12)) * batch

    def one(names, per_amp=None):
        """launch-weighted totals over the kernels whose names contain any of
        `names`; per_amp = algorithmic bytes per amplitude by name (None: 16 B
        per direction the counters show)"""
        n = 0
        f_tot = w_tot = alg_tot = 0.0
        for kname in names:
            fsel = fe[fe.Kernel_Name.str.contains(kname, regex=False)]["Counter_Value"]
            wsel = wr[wr.Kernel_Name.str.contains(kname, regex=False)]["Counter_Value"]
            if not len(fsel) or not len(wsel):
                continue
            f, w = fsel.mean() * 1024, wsel.mean() * 1024
            hbm = 2 * f + w
            if per_amp and kname in per_amp:
                a = per_amp[kname] * amps
            else:
                a = 16.0 * (int(2 * f > 0.01 * hbm) + int(w > 0.01 * hbm)) * amps
            k = len(fsel)
            n += k
            f_tot += f * k
            w_tot += w * k
            alg_tot += a * k
        if not n:
            return None
        hbm = (2 * f_tot + w_tot) / n
        return {"kernel": " + ".join(names), "launches": n, "fetch_bytes_raw": f_tot / n,
                "write_bytes": w_tot / n, "hbm_bytes_per_launch": hbm,
                "algorithmic_bytes_per_launch": alg_tot / n,
                "ratio_to_algorithmic": hbm / (alg_tot / n)}

    if "--config c5" in bench_args:
        # one L=34 state over virtual shards: every pass kernel of the run (slice
        # kicks, the fused kick+exchange, the K-D-K) against the bench line's
        # own algorithmic pass bytes (printed by the same command), per period
        line = None
        with open(f"{prof}/fetch.log") as fh:
            for ln in fh:
                if ln.startswith("{"):
                    line = json.loads(ln)
        periods = line["steps"] * (line["config"]["tf"] - 1)
        alg = line["roofline"]["algorithmic_bytes_per_period"] * periods
        hbm = 0.0
        n = 0
        for kname in ("dtc_kdk_pass", "dtc_kick_pass", "dtc_kick_swap_pass"):
            fsel = fe[fe.Kernel_Name.str.contains(kname, regex=False)]["Counter_Value"]
            wsel = wr[wr.Kernel_Name.str.contains(kname, regex=False)]["Counter_Value"]
            hbm += 2 * fsel.sum() * 1024 + wsel.sum() * 1024
            n += len(fsel)
        res["lo_pass"] = {"kernel": "C5 pass kernels per period (dtc_kdk_pass, dtc_kick_pass, "
                                    "dtc_kick_swap_pass)", "launches": n, "periods": periods,
                          "hbm_bytes_per_launch": hbm / periods,
                          "algorithmic_bytes_per_launch": alg / periods,
                          "ratio_to_algorithmic": hbm / alg, "unit": "per period"}
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)
        print(json.dumps(res, indent=1))
        return
    # the K-D-K passes as the bench line aggregates them: dtc_kdk_pass /
    # dtc_kdk_pass3 (32 B per amplitude) and the dual forward+echo-start
    # dtc_kdk_dual (48 B: one read, two stores)
    for key, names, per_amp in (
            ("lo_pass", ("dtc_kdk_pass", "dtc_kdk_dual"), {"dtc_kdk_pass": 32.0, "dtc_kdk_dual": 48.0}),
            ("kdk_single", ("dtc_kdk_pass",), {"dtc_kdk_pass": 32.0}),
            ("kdk_dual", ("dtc_kdk_dual",), {"dtc_kdk_dual": 48.0}),
            ("hi_pass", ("dtc_kick_pass",), None),
            # (the light-cone ends read the state once and store only their
            # per-tile partials: 16 B per amplitude whatever the counters show)
            ("lightcone_pass", ("dtc_lc_final",), {"dtc_lc_final": 16.0}),
            ("lightcone_wide_pass", ("dtc_lcw2_final", "dtc_lcw_final"),
             {"dtc_lcw2_final": 16.0, "dtc_lcw_final": 16.0}),
            ("lightcone_12site_pass", ("dtc_lcw3_final",), {"dtc_lcw3_final": 16.0})):
        r = one(names, per_amp)
        if r:
            res[key] = r
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]),
         sys.argv[5] if len(sys.argv) > 5 else "")
