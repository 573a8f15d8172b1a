#!/bin/bash
# Development A/B of engine environment switches on any bench config (GPU box,
# repo root): bench.py <args> once per setting, value + roofline kernel rate.
# Usage: bash tools/ab_config.sh <tag> "<bench args>" "VAR=a" "VAR=b" ...
set -o pipefail
TAG=$1; ARGS=$2; shift 2
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
i=0
for setting in "$@"; do
  i=$((i+1)); n=${TAG}_$i
  ( export $setting; timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > $O/abc_$n.json 2> $O/abc_$n.err ) || { echo "$setting failed"; tail -3 $O/abc_$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/abc_$n.json')); r=d['roofline']; k=d.get('kernels',{}); print('$setting', '$ARGS', round(d['value'],1), round(r['achieved']), round(r.get('avg_launch_ms') or 0, 4), 'kick', round((k.get('kick_pass') or {}).get('avg_ms') or 0, 3))"
done
