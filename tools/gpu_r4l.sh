# r4l: the full GPU suite with the 12-site light-cone end; SQ counters of the
# C2 kernels (dtc_lcw3_final's instruction mix)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r4l_gputest.txt 2>&1; rc=$?
tail -8 $O/r4l_gputest.txt
[ $rc -le 1 ] || exit $rc
bash tools/pmc_sq.sh r4l || exit 1
python tools/sq_table.py gpurun_out/pmc_r4l lcw3 lcw2 kdk_pass lc_final > $O/r4l_sq_table.md || exit 1
cat $O/r4l_sq_table.md
exit $rc
