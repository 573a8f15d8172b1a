#!/bin/bash
# round 6 call c: column-pass probe, the new parity tests, SQ counters of the C2 kernels
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/gpu_run.sh r6c exec:tile13_kdk_probe "tests:split_invariance or device_kd_dual or device_dual_pass or energy_sums or c3_schedule" || exit 1
B=64 bash tools/pmc_sq.sh r6c || exit 1
echo r6c done
