#!/bin/bash
# Every bench.py config once (GPU box, repo root) -> gpurun_out/<tag>_<config>_bench.json,
# plus a rocprofv3 --kernel-trace --stats of the energy line (its roofline kernels).
# Usage: bash tools/measure_configs.sh <tag> [configs...]
set -o pipefail
TAG=$1; shift
CONFIGS=${@:-c3 c4 energy ctrl c5}
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
for c in $CONFIGS; do
  timeout -k 10 300 python -u bench.py --config $c > $O/${TAG}_${c}_bench.json 2> $O/${TAG}_${c}_bench.err || { echo "$c failed"; tail -5 $O/${TAG}_${c}_bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/${TAG}_${c}_bench.json')); r=d.get('roofline',{}); print('$c', round(d['value'],2), d['unit'], round(r.get('achieved',0)), r.get('avg_launch_ms'))"
done
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${TAG}_energy -o kt -- python $R/bench.py --config energy --no-cpu-baseline > $O/prof_${TAG}_energy.log 2>&1 || { echo "energy trace failed"; exit 1; }
echo configs done
