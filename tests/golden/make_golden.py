"""Extract the reference's committed data into small JSON fixtures.

Run once in the build container (needs /root/reference, read as data only):
    python tests/golden/make_golden.py
Outputs (committed; the GPU box never reads /root/reference):
  disorder.json     first rows of hs_L{4,6,20}.csv / phis_L{4,6,20}.csv
                    (input files read by fast.py:66-74)
  aer_autocorr.json 1024-shot Aer outputs committed by the reference
                    (autocorr_data_L4/, autocorr_data_L20_polarization/,
                    autocorr_data_L20_circular-polarization/,
                    controlled-autocorr_data_L20/)
  gate_counts.json  every gate_counts_*aer_simulator*.csv (fast.py:193-197)
  adaptive.json     per-instance adaptive-g histories (g, echo, forward per t) of
                    autocorr_data_L4/*realtime_adaptive* and
                    controlled-autocorr_data_L20/*optimization*
  envelopes.json    series + envelope columns of the *_with_envelopes.csv files
                    and of the controlled-g optimisation CSV
Nothing here is source code of the reference: only numeric columns.
"""
from __future__ import annotations

import glob
import json
import os
import re

import pandas as pd

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def disorder():
    out = {}
    for L, rows in ((4, 1), (6, 1), (20, 16)):
        hs = pd.read_csv(f"{REF}/hs_L{L}.csv", comment="#", header=0)
        ph = pd.read_csv(f"{REF}/phis_L{L}.csv", comment="#", header=0)
        out[f"L{L}"] = {
            "source": [f"hs_L{L}.csv", f"phis_L{L}.csv"],
            "hs": hs.iloc[:rows].values.tolist(),
            "phis": ph.iloc[:rows].values.tolist(),
        }
    return out


def aer_autocorr():
    cases = []

    def add(path, name, cfg, cols):
        df = pd.read_csv(f"{REF}/{path}")
        cases.append({
            "name": name,
            "file": path,
            "config": cfg,
            "time": df["time"].tolist(),
            "columns": {k: df[v].tolist() for k, v in cols.items()},
        })

    l4 = "autocorr_data_L4/autocorr_data_vacuum_realtime_adaptive_g0.84_L4_inst1_randomphi1_delta0.0_amplitude1.0_noise0.05_usenoise1_target1.0_gain{}.csv"
    for gain in ("0.01", "0.05"):
        add(l4.format(gain), f"L4_ctrl_standard_gain{gain}",
            {"L": 4, "g": 0.84, "noise": 0.05, "t_offset": 1, "polarization": "x",
             "initial_state": "vacuum", "inst_row": 0, "shots": 1024},
            {"fwd": "av_autocorr_standard", "echo": "av_autocorr_echo_standard",
             "fwd_adaptive": "av_autocorr_adaptive", "echo_adaptive": "av_autocorr_echo_adaptive",
             "g_adaptive": "av_g_values"})
    circ = ("autocorr_data_L20_circular-polarization/autocorr_data_vacuum_g0.97_L20_inst1_"
            "randomphi1_delta0.0_amplitude1.0_noise0.05_usenoise1_pol{}_with_envelopes.csv")
    for pol in ("x", "y", "circular_left", "circular_right"):
        add(circ.format(pol), f"L20_circ_{pol}",
            {"L": 20, "g": 0.97, "noise": 0.05, "t_offset": 0, "polarization": pol,
             "circular_frequency": 1.0, "initial_state": "vacuum", "inst_row": 0, "shots": 1024},
            {"fwd": "av_autocorr", "echo": "av_autocorr_echo"})
    pold = ("autocorr_data_L20_polarization/autocorr_data_vacuum_g0.97_L20_inst1_"
            "randomphi1_delta0.0_amplitude1.0_noise0.05_usenoise1_pol{}_with_envelopes.csv")
    for pol in ("x", "y", "xy", "yx"):
        add(pold.format(pol), f"L20_pol_{pol}",
            {"L": 20, "g": 0.97, "noise": 0.05, "t_offset": 0, "polarization": pol,
             "initial_state": "vacuum", "inst_row": 0, "shots": 1024},
            {"fwd": "av_autocorr", "echo": "av_autocorr_echo"})
    ctrl = ("controlled-autocorr_data_L20/autocorr_data_vacuum_realtime_adaptive_optimization_"
            "iter5_g0.84_L20_inst1_randomphi1_delta0.0_amplitude1.0_noise0.05_usenoise1_"
            "target1.0_gain0.01.csv")
    for g, tag in ((0.97, "g97"), (0.84, "g84")):
        add(ctrl, f"L20_ctrl_standard_{tag}",
            {"L": 20, "g": g, "noise": 0.05, "t_offset": 1, "polarization": "x",
             "initial_state": "vacuum", "inst_row": 0, "shots": 1024},
            {"fwd": f"av_autocorr_standard_{tag}", "echo": f"av_autocorr_echo_standard_{tag}"})
    return cases


def gate_counts():
    out = []
    pat = re.compile(r"gate_counts_t(\d+)_(forward|echo)_opt0_aer_simulator_.*_(iqm|polarization)\.csv")
    for path in sorted(glob.glob(f"{REF}/*/gate_counts_t*_aer_simulator_*.csv")):
        m = pat.search(os.path.basename(path))
        if not m:
            continue
        folder = os.path.basename(os.path.dirname(path))
        df = pd.read_csv(path)
        out.append({
            "folder": folder,
            "t": int(m.group(1)),
            "echo": m.group(2) == "echo",
            "counts": {str(r.gate): int(r.count) for r in df.itertuples()},
        })
    return out


L4_ADAPT = ("autocorr_data_L4/autocorr_data_vacuum_realtime_adaptive_g0.84_L4_inst1_randomphi1_"
            "delta0.0_amplitude1.0_noise0.05_usenoise1_target1.0_gain{}.csv")
L20_OPT = ("controlled-autocorr_data_L20/autocorr_data_vacuum_realtime_adaptive_optimization_"
           "iter5_g0.84_L20_inst1_randomphi1_delta0.0_amplitude1.0_noise0.05_usenoise1_"
           "target1.0_gain0.01.csv")


def adaptive():
    out = []
    for gain in ("0.01", "0.05"):
        df = pd.read_csv(f"{REF}/{L4_ADAPT.format(gain)}")
        out.append({"name": f"L4_realtime_gain{gain}", "file": L4_ADAPT.format(gain),
                    "config": {"L": 4, "g": 0.84, "noise": 0.05, "t_offset": 1,
                               "target": 1.0, "gain": float(gain), "g_min": 0.84},
                    "g": df["g_history_inst1"].tolist(),
                    "echo": df["echo_adaptive_inst1"].tolist(),
                    "fwd": df["forward_adaptive_inst1"].tolist()})
    df = pd.read_csv(f"{REF}/{L20_OPT}")
    out.append({"name": "L20_optimization", "file": L20_OPT, "columns": list(df.columns),
                "config": {"L": 20, "g": 0.84, "noise": 0.05, "t_offset": 1, "target": 1.0,
                           "g_min": 0.84, "g_max": 1.0},
                "g": df["g_history_inst1"].tolist(),
                "echo": df["echo_adaptive_inst1"].tolist(),
                "fwd": df["forward_adaptive_inst1"].tolist()})
    return out


def envelopes():
    out = []
    pol = glob.glob(f"{REF}/autocorr_data_L20_*polarization/autocorr_data_vacuum_*_pol*_with_envelopes.csv")
    for path in sorted(pol):
        df = pd.read_csv(path)
        rel = os.path.relpath(path, REF)
        for sig, up, lo in (("av_autocorr", "forward_upper_env", "forward_lower_env"),
                            ("av_autocorr_echo", "echo_upper_env", "echo_lower_env"),
                            ("sqrt_av_autocorr_echo", "sqrt_echo_upper_env",
                             "sqrt_echo_lower_env")):
            out.append({"file": rel, "variant": "polarization", "window": 3,
                        "signal": df[sig].tolist(), "upper": df[up].tolist(),
                        "lower": df[lo].tolist()})
    df = pd.read_csv(f"{REF}/{L20_OPT}")
    for sig, tag in (("av_autocorr_adaptive", "adaptive_forward"),
                     ("av_autocorr_standard_g84", "g84_forward"),
                     ("av_autocorr_standard_g97", "g97_forward"),
                     ("av_autocorr_echo_adaptive", "adaptive_echo"),
                     ("av_autocorr_echo_standard_g84", "g84_echo"),
                     ("av_autocorr_echo_standard_g97", "g97_echo")):
        out.append({"file": L20_OPT, "variant": "controlled", "window": 3,
                    "signal": df[sig].tolist(), "upper": df[f"upper_env_{tag}"].tolist(),
                    "lower": df[f"lower_env_{tag}"].tolist()})
    return out


def main():
    with open(os.path.join(OUT, "disorder.json"), "w") as f:
        json.dump(disorder(), f, indent=1)
    with open(os.path.join(OUT, "aer_autocorr.json"), "w") as f:
        json.dump(aer_autocorr(), f, indent=1)
    with open(os.path.join(OUT, "gate_counts.json"), "w") as f:
        json.dump(gate_counts(), f, indent=0)
    with open(os.path.join(OUT, "adaptive.json"), "w") as f:
        json.dump(adaptive(), f, indent=1)
    with open(os.path.join(OUT, "envelopes.json"), "w") as f:
        json.dump(envelopes(), f, indent=0)
    print("wrote fixtures to", OUT)


if __name__ == "__main__":
    main()
