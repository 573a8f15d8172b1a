#!/bin/bash
# Collect PMC counter sets (one rocprofv3 pass each) on a short bench run.
# Usage: bash tools/pmc_run.sh <tag> "<counters pass 1>" "<counters pass 2>" ...
set -o pipefail
TAG=$1; shift
R=$(pwd); O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
i=0
for set in "$@"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $set -T --output-format csv -d $O -o p$i -- python $R/bench.py --steps 1 --warmup 0 --strong-total 0 --batch 64 --no-cpu-baseline > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
