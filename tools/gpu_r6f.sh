#!/bin/bash
# round 6 call f: 13-site pass with the conflict-free slot maps (13-bit tile, lcw3),
# RecScalar (product) / RecRegs records, against the 12 / 8 split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/ab_libs.sh r6f base devlib/t13regs.so || exit 1
bash tools/ab_env.sh r6f DTC_NO_SPLIT13=1 DTC_AB=0 || exit 1
echo r6f done
