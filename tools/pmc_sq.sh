#!/bin/bash
# SQ-level counters of the C2 pass kernels (one rocprofv3 pass per counter
# set; counters list saved first).  Usage: bash tools/pmc_sq.sh <tag>
set -o pipefail
TAG=$1
R=$(pwd); O=$R/gpurun_out/pmc_$TAG
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
i=0
for set in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM" \
  "GRBM_GUI_ACTIVE GRBM_COUNT" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $O -o p$i -- python $R/bench.py --steps 1 --warmup 0 --strong-total 0 --batch ${B:-64} --no-cpu-baseline $BENCH_ARGS > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/p$i.log; exit 1; }
done
echo done
