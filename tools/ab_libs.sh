#!/bin/bash
# Development A/B of kernel build variants (not the product): bench.py (C2, or
# $BENCH_ARGS, e.g. "--config energy") under
# rocprofv3 --kernel-trace --stats once per library.  Usage (GPU box, repo root):
#   bash tools/ab_libs.sh <tag> base devlib/libA.so devlib/libB.so ...   (base = lib/libdtc_hip.so)
set -o pipefail
TAG=$1; shift
R=$(pwd); O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
i=0
for lib in "$@"; do
  i=$((i+1)); n=${TAG}_$i
  if [ "$lib" = base ]; then unset DTC_LIB; else export DTC_LIB=$R/$lib; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ab_$n -o kt -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $O/ab_$n.json 2> $O/ab_$n.err || { echo "$lib failed"; exit 1; }
  python - "$O/ab_$n" "$lib" <<'PY'
import json, sys, pandas as pd
d = json.load(open(sys.argv[1] + ".json"))
k = pd.read_csv(sys.argv[1] + "/kt_kernel_stats.csv")
k = k[k.Name.str.contains("kdk|lcw|lc_final|pass13|kick_swap|kick_pass")]
print(sys.argv[2], round(d["value"]), round(d["roofline"]["achieved"]),
      " ".join(f"{r.Name.split('dtc_')[-1].split('(')[0].replace(' ', '')}={r.AverageNs / 1e6:.4f}" for r in k.itertuples()))
PY
done
