#!/bin/bash
# r3zw: scheduler-option builds (max-ilp, AMDGPU register trackers) against the
# default build on C2 and energy, alternating (development A/B, not the product)
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  bash tools/ab_libs.sh r3zw_c2_$i base devlib/libdtc_ilp.so devlib/libdtc_trk.so >> gpurun_out/r3zw_ab.txt 2>&1 || exit 1
done
BENCH_ARGS="--config energy" bash tools/ab_libs.sh r3zw_en base devlib/libdtc_ilp.so devlib/libdtc_trk.so >> gpurun_out/r3zw_ab.txt 2>&1 || exit 1
