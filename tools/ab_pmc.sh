#!/bin/bash
# WRITE_SIZE of the C2 pass kernels under one engine environment setting (GPU
# box, repo root): the spill check of a kernel variant.  Usage:
#   bash tools/ab_pmc.sh <tag> "VAR=value"
set -o pipefail
TAG=$1; SETTING=$2
R=$(pwd); O=$R/gpurun_out/pmcw_$TAG; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
( export $SETTING; timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O -o w -- python $R/bench.py --steps 1 --warmup 0 --strong-total 0 --batch 256 --no-cpu-baseline > $O/w.log 2>&1 ) || { echo "pmc pass failed"; tail -5 $O/w.log; exit 1; }
python - "$O" "$SETTING" <<'PY'
import sys, pandas as pd
d = pd.read_csv(sys.argv[1] + "/w_counter_collection.csv")
d = d[d.Kernel_Name.str.contains("kdk|lc_final")]
alg = 16.0 * (1 << 20) * 256
g = (d.groupby("Kernel_Name").Counter_Value.mean() * 1024 / alg).round(4)
print(sys.argv[2], " ".join(f"{k.split('dtc::')[1].split('(')[0]}={v}" for k, v in g.items()))
PY
