#!/bin/bash
# One GPU call's worth of C2 evidence (GPU box, repo root):
#   bench line (default C2) -> gpurun_out/<tag>_bench.json
#   rocprofv3 --kernel-trace --stats of the same command -> gpurun_out/prof_<tag>/
#   PMC FETCH_SIZE / WRITE_SIZE passes at the bench's batch -> gpurun_out/<tag>_pmc.json
# Usage: bash tools/measure_c2.sh <tag> [extra bench args]
set -o pipefail
TAG=$1; shift
R=$(pwd); O=$R/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u bench.py "$@" > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; tail -5 $O/${TAG}_bench.err; exit 1; }
cat $O/${TAG}_bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o kt -- python $R/bench.py --no-cpu-baseline "$@" > $O/prof_${TAG}_kt.log 2>&1 || { echo "kernel trace failed"; tail -5 $O/prof_${TAG}_kt.log; exit 1; }
cd $R
bash tools/pmc_traffic.sh $TAG 1024 || exit 1
echo measure done
