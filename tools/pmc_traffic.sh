#!/bin/bash
# HBM traffic of the pass kernels of one bench config (MI355X_MICROARCH.md
# §HBM: separate rocprofv3 --pmc passes for FETCH_SIZE and WRITE_SIZE,
# FETCH_SIZE doubled for gfx950) -> gpurun_out/<tag><suffix>.json via
# tools/pmc_summary.py; copy it to profiles/ to make the bench line cite it.
# Usage (GPU box, repo root): bash tools/pmc_traffic.sh <tag> [batch]
#   batch: states per launch, default 1024 = the C2/C3 line's (the summary is
#   only used by a line of the same batch)
#   BENCH_ARGS="--config c3" SUFFIX=_pmc_c3          C3 (device-like noise)
#   BENCH_ARGS="--config energy" SUFFIX=_pmc_energy  energy path (batch 1024)
#   BENCH_ARGS="--config c4" SUFFIX=_pmc_c4 L=28 ... 32   C4 (32 instances: one
#   launch holds the 32 L=28 states)
set -o pipefail
TAG=$1; B=${2:-1024}; L=${L:-20}
R=$(pwd); O=$R/gpurun_out/pmc_$TAG${SUFFIX}
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  timeout -s KILL 180 rocprofv3 --pmc $c --output-format csv -d $O -o $n -- python $R/bench.py --steps 1 --warmup 0 --strong-total 0 --batch $B --no-cpu-baseline $BENCH_ARGS > $O/$n.log 2>&1 || { echo "$c pass failed"; tail -5 $O/$n.log; exit 1; }
done
python $R/tools/pmc_summary.py $O $R/gpurun_out/${TAG}${SUFFIX:-_pmc}.json $B $L "$BENCH_ARGS"
