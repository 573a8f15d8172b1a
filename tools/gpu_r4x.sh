# r4x: end-of-round HEAD re-profile (device dual pass in the product): C2 (bench +
# kernel stats + PMC), C4 / C3 / energy each with bench, kernel stats and PMC
# traffic at the line's own batch; ctrl and C5 bench lines; the GPU suite.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
bash tools/measure_c2.sh r4x || exit 1
export TMPDIR=/tmp
for c in c4 c3 energy; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/r4x_${c}_bench.json 2> $O/r4x_${c}_bench.err || { tail -5 $O/r4x_${c}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/r4x_${c}_bench.json')); r=d['roofline']; print('$c', round(d['value'], 2), round(r['achieved']), r.get('avg_launch_ms'), d.get('kernels'))"
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r4x_$c -o kt -- python $R/bench.py --config $c --no-cpu-baseline --steps 2 --warmup 1 > $R/$O/prof_r4x_${c}.log 2>&1) || { echo "$c trace failed"; exit 1; }
done
L=28 BENCH_ARGS="--config c4" SUFFIX=_pmc_c4 bash tools/pmc_traffic.sh r4x 32 || exit 1
BENCH_ARGS="--config c3" SUFFIX=_pmc_c3 bash tools/pmc_traffic.sh r4x 1024 || exit 1
BENCH_ARGS="--config energy" SUFFIX=_pmc_energy bash tools/pmc_traffic.sh r4x 1024 || exit 1
for c in ctrl c5; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $O/r4x_${c}_bench.json 2> $O/r4x_${c}_bench.err || { tail -5 $O/r4x_${c}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/r4x_${c}_bench.json')); print('$c', round(d['value'], 2))"
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r4x_smoke.txt 2>&1 || { cat $O/r4x_smoke.txt; exit 1; }
tail -1 $O/r4x_smoke.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r4x_gputest.txt 2>&1; rc=$?
tail -6 $O/r4x_gputest.txt
[ $rc -le 1 ] || exit $rc
echo ok
