# r4i: fully coupled L=28 against the C oracle (C4 engine path and the C5
# sharded pipeline with 8 virtual shards).  The oracle's sweep is one long
# host call: a heartbeat line every minute shows the run is alive.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
(while true; do sleep 60; echo "heartbeat $(date +%T)"; done) &
HB=$!
timeout -k 10 900 python -u -m pytest tests/test_gpu_l28_oracle.py -m gpu -v --timeout 800 --timeout-method thread --durations=5 > $O/r4i_tests.txt 2>&1; rc=$?
kill $HB
tail -15 $O/r4i_tests.txt
exit $rc
