# r4p: coupled L=28 / L=30 parity against the C oracle (C4 and C5 paths)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) &
HB=$!
timeout -k 10 900 python -u -m pytest tests/test_gpu_l28_oracle.py -m gpu -v --timeout 800 --timeout-method thread --durations=5 > $O/r4p_tests.txt 2>&1; rc=$?
kill $HB
tail -14 $O/r4p_tests.txt
exit $rc
