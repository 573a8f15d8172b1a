# r4b: dtc_lcw2_final parity, the loopback real-rank exchange, the fused
# kick+exchange (C5 one GPU), then same-box A/B vs the six-re-layout light
# cone (devlib/dev_r4.so = DEV build of the same source; DTC_LC_TPB=-1 keeps
# dtc_lcw_final) and the 13-bit tile pattern study
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "lcw2 or light_cone or matches_oracle or random_state" > $O/r4b_tests.txt 2>&1 || { tail -40 $O/r4b_tests.txt; exit 1; }
tail -3 $O/r4b_tests.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_golden.py > $O/r4b_golden.txt 2>&1 || { tail -30 $O/r4b_golden.txt; exit 1; }
tail -2 $O/r4b_golden.txt
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py -k "loopback or inplace or exchange_slice" > $O/r4b_sharded.txt 2>&1 || { tail -40 $O/r4b_sharded.txt; exit 1; }
tail -8 $O/r4b_sharded.txt
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4b_new_$i.json 2> $O/r4b_new_$i.err || exit 1
  DTC_LIB=$GRAFT_REPO_ROOT/devlib/dev_r4.so DTC_LC_TPB=-1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4b_old_$i.json 2> $O/r4b_old_$i.err || exit 1
  python - $O/r4b_new_$i.json $O/r4b_old_$i.json <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    k = d.get("kernels", {})
    print(f, round(d["value"]), {n: (round(v.get("avg_ms"), 4) if isinstance(v, dict) and v.get("avg_ms") else None) for n, v in k.items()})
PY
done
timeout -k 10 120 ./tools/tile13_bench > $O/r4b_tile13.txt 2>&1 || exit 1
cat $O/r4b_tile13.txt
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r4b -o kt -- python $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/prof_r4b.log 2>&1 || exit 1
echo ok
