# r4d: the full GPU suite at the candidate build (additive slots without LDS
# op merging, dual forward+echo passes, lcw2, fused C5 kick+exchange), then
# same-box A/B: product vs DTC_NO_DUAL, and vs the XOR-slot build with merging
# (devlib/dev_xor.so), on C2 and energy; C5 at L=34 (one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
summ() {
python - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    k = d.get("kernels", {})
    print(f.split("/")[-1], round(d["value"]), {n: (round(v.get("avg_ms"), 4) if isinstance(v, dict) and v.get("avg_ms") else None) for n, v in k.items()})
PY
}
D=$GRAFT_REPO_ROOT/devlib
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4d_new_$i.json 2> $O/r4d_new_$i.err || exit 1
  DTC_NO_DUAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4d_nodual_$i.json 2> $O/r4d_nodual_$i.err || exit 1
  DTC_LIB=$D/dev_xor.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4d_xor_$i.json 2> $O/r4d_xor_$i.err || exit 1
  DTC_LIB=$D/dev_xor.so DTC_NO_DUAL=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4d_xornodual_$i.json 2> $O/r4d_xornodual_$i.err || exit 1
  summ $O/r4d_new_$i.json $O/r4d_nodual_$i.json $O/r4d_xor_$i.json $O/r4d_xornodual_$i.json
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --config energy --no-cpu-baseline --steps 3 --warmup 1 > $O/r4d_en_new_$i.json 2> $O/r4d_en_new_$i.err || exit 1
  DTC_LIB=$D/dev_xor.so timeout -k 10 200 python bench.py --config energy --no-cpu-baseline --steps 3 --warmup 1 > $O/r4d_en_xor_$i.json 2> $O/r4d_en_xor_$i.err || exit 1
  summ $O/r4d_en_new_$i.json $O/r4d_en_xor_$i.json
done
timeout -k 10 400 python bench.py --config c5 --no-cpu-baseline --steps 2 --warmup 1 > $O/r4d_c5.json 2> $O/r4d_c5.err || exit 1
python -c "import json; d=json.load(open('$O/r4d_c5.json')); print('c5', d['value'], d.get('period_ms'), d.get('pass_ms_per_period'), d.get('exchange',{}).get('per_period_ms'))"
timeout -k 10 120 ./tools/tile13_bench > $O/r4d_tile13.txt 2>&1 || exit 1
for i in 1 2; do DTC_LIB=$D/lcw3.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4d_lcw3_$i.json 2> $O/r4d_lcw3_$i.err || exit 1; summ $O/r4d_lcw3_$i.json; done
head -12 $O/r4d_tile13.txt
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r4d -o kt -- python $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/prof_r4d.log 2>&1 || exit 1
cd $R && python - <<'PY'
import glob, pandas as pd
f = glob.glob("gpurun_out/prof_r4d/**/kt_kernel_stats.csv", recursive=True)[0]
k = pd.read_csv(f)
print(k[["Name", "Calls", "AverageNs", "Percentage"]].head(14).to_string())
PY
# the suite last: a plain test failure (rc 1) is reported, anything else ends here
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/r4d_gputest.txt 2>&1; rc=$?
tail -8 $O/r4d_gputest.txt
[ $rc -le 1 ] || exit $rc
echo ok
