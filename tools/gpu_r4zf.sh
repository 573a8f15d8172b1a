# r4zf: HEAD confirmation after the container rebuild (kick-only measure-only end at three
# per CU in the product): C2 bench + kernel stats + PMC, C3 bench + kernel stats, ctrl,
# smoke, and the full GPU suite on the same binary.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
bash tools/measure_c2.sh r4zf || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/r4zf_c3_bench.json 2> $O/r4zf_c3_bench.err || { tail -5 $O/r4zf_c3_bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/r4zf_c3_bench.json')); print('c3', round(d['value']))"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r4zf_c3 -o kt -- python $R/bench.py --config c3 --no-cpu-baseline --steps 2 --warmup 1 > $R/$O/prof_r4zf_c3.log 2>&1) || { echo "c3 trace failed"; exit 1; }
timeout -k 10 300 python -u bench.py --config ctrl --no-cpu-baseline > $O/r4zf_ctrl_bench.json 2> $O/r4zf_ctrl_bench.err || { tail -5 $O/r4zf_ctrl_bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/r4zf_ctrl_bench.json')); print('ctrl', round(d['value']))"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r4zf_smoke.txt 2>&1 || { cat $O/r4zf_smoke.txt; exit 1; }
tail -1 $O/r4zf_smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r4zf_gputest.txt 2>&1; rc=$?
tail -6 $O/r4zf_gputest.txt
[ $rc -le 1 ] || exit $rc
echo ok
