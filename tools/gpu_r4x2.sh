# r4x2: the final binary (device dual pass also for general kicks): C2 and C3
# bench lines, ctrl, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 300 python -u bench.py > $O/r4x2_bench.json 2> $O/r4x2_bench.err || { tail -5 $O/r4x2_bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/r4x2_bench.json')); print('c2', round(d['value']), round(d['roofline']['achieved']), d['roofline']['traffic_source'])"
for c in c3 ctrl; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline > $O/r4x2_${c}_bench.json 2> $O/r4x2_${c}_bench.err || { tail -5 $O/r4x2_${c}_bench.err; exit 1; }
  python -c "import json; d=json.load(open('$O/r4x2_${c}_bench.json')); print('$c', round(d['value']))"
done
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r4x2_smoke.txt 2>&1 || { cat $O/r4x2_smoke.txt; exit 1; }
tail -1 $O/r4x2_smoke.txt
