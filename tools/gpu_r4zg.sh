# r4zg: the remaining bench lines at HEAD (C4, energy, C5 on one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
for c in c4 energy c5; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $O/r4zg_${c}_bench.json 2> $O/r4zg_${c}_bench.err || { tail -5 $O/r4zg_${c}_bench.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/r4zg_${c}_bench.json').read().strip().splitlines()[-1]); print('$c', round(d['value'], 2))"
done
echo ok
