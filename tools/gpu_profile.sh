#!/bin/bash
# Bench + rocprofv3 kernel-trace/stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE).
# Usage (on the GPU box, from the repo root): bash tools/gpu_profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r1}; shift
R=$(pwd); O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 python $R/bench.py "$@" > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed $?"; exit 1; }
cat $O/bench_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$TAG -o kt -- python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $O/prof_${TAG}_kt.log 2>&1 || { echo "kt failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d $O/prof_$TAG -o fetch -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/prof_${TAG}_fetch.log 2>&1 || { echo "fetch failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d $O/prof_$TAG -o write -- python $R/bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $O/prof_${TAG}_write.log 2>&1 || { echo "write failed $?"; exit 1; }
find $O/prof_$TAG -type f | head -50
