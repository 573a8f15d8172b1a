#!/bin/bash
# Development: the C2 line's batch schedule (DTC_PRINT_SCHED, a DEV build) next
# to its kernel trace, for matching launch durations to schedule entries.
# Usage (GPU box, repo root): [CMD="tools/c2_variant.py --noise 0"] bash tools/sched_trace.sh <tag> <devlib.so> [VAR=v ...]
set -o pipefail
TAG=$1; LIB=$2; shift 2
R=$(pwd); O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
( export DTC_LIB=$R/$LIB DTC_PRINT_SCHED=1; for s in "$@"; do export "$s"; done
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/st_$TAG -o kt -- python $R/${CMD:-bench.py --steps 1 --warmup 0 --no-cpu-baseline} > $O/st_$TAG.json 2> $O/st_$TAG.sched ) || { echo "sched trace failed"; tail -5 $O/st_$TAG.sched; exit 1; }
cat $O/st_$TAG.json
