#!/bin/bash
# Development: sample the GPU's power and clocks (rocm-smi, read-only) every
# ~0.2 s while a command runs.  Usage (GPU box): bash tools/power_sample.sh <tag> <cmd...>
TAG=$1; shift
O=gpurun_out; mkdir -p $O
( while true; do echo "T $(date +%s.%N)"; rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Power|sclk|mclk|fclk"; sleep 0.2; done ) > $O/pw_$TAG.txt &
SP=$!
timeout -k 10 300 "$@" > $O/pw_$TAG.out 2>&1; rc=$?
kill $SP
exit $rc
