#!/bin/bash
# r3zv: energy K-D-K pass3 with the pre-kick X compiled out (MC 4): energy
# parity, then alternating energy benches against the previous build.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_energy.py > gpurun_out/r3zv_tests.txt 2>&1 || exit 1
for i in 1 2; do
  BENCH_ARGS="--config energy" bash tools/ab_libs.sh r3zv_$i devlib/libdtc_hip_base.so base >> gpurun_out/r3zv_ab.txt 2>&1 || exit 1
done
