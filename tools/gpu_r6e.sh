#!/bin/bash
# round 6 call e: 13-site pass variants (records, kick variants) and SQ counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/ab_libs.sh r6e base devlib/t13var0.so devlib/t13regs.so devlib/t13var0regs.so || exit 1
B=64 bash tools/pmc_sq.sh r6e || exit 1
echo r6e done
