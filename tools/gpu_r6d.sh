#!/bin/bash
# round 6 call d: the 13 / 7 split -- parity tests, then a same-box A/B against the 12 / 8 split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
O=gpurun_out; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "split13 or headline or split_invariance or lcw3 or dual_pass or echo_light or apply_periods" > $O/r6d_gputest.txt 2>&1; rc=$?
tail -5 $O/r6d_gputest.txt
[ $rc -le 1 ] || exit $rc
bash tools/ab_env.sh r6d DTC_AB=0 DTC_NO_SPLIT13=1 DTC_AB=0 DTC_NO_SPLIT13=1 || exit 1
echo r6d done
