# r4n: final HEAD measurement -- C2 bench line (with the CPU baseline),
# rocprof kernel stats and PMC traffic of the same command (tools/measure_c2.sh),
# the ctrl line (its echo chains end in the new light cone), smoke, GPU suite
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
bash tools/measure_c2.sh r4n || exit 1
timeout -k 10 400 python -u bench.py --config ctrl --no-cpu-baseline > $O/r4n_ctrl_bench.json 2> $O/r4n_ctrl_bench.err || { tail -5 $O/r4n_ctrl_bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/r4n_ctrl_bench.json')); print('ctrl', round(d['value'], 1))"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r4n_smoke.txt 2>&1 || { cat $O/r4n_smoke.txt; exit 1; }
cat $O/r4n_smoke.txt | tail -2
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r4n_gputest.txt 2>&1; rc=$?
tail -4 $O/r4n_gputest.txt
exit $rc
