#!/bin/bash
# HBM traffic of the C2 pass kernels (MI355X_MICROARCH.md §HBM: separate
# rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE, FETCH_SIZE doubled for
# gfx950) -> profiles/<tag>_pmc.json via tools/pmc_summary.py.
# Usage (GPU box, repo root): bash tools/pmc_traffic.sh <tag> [batch]
# (BENCH_ARGS="--config energy" SUFFIX=_pmc_energy: the energy path's passes)
set -o pipefail
TAG=$1; B=${2:-64}
R=$(pwd); O=$R/gpurun_out/pmc_$TAG${SUFFIX}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $O -o $n -- python $R/bench.py --steps 1 --warmup 0 --strong-total 0 --batch $B --no-cpu-baseline $BENCH_ARGS > $O/$n.log 2>&1 || { echo "$c pass failed"; tail -5 $O/$n.log; exit 1; }
done
python $R/tools/pmc_summary.py $O $R/gpurun_out/${TAG}${SUFFIX:-_pmc}.json $B 20
