# r4c: the loopback real-rank exchange and the fused kick+exchange (C5 one
# GPU) tests; same-box A/B of dtc_lcw2_final vs dtc_lcw_final (DEV build,
# DTC_LC_TPB=-1) and of the additive half-tile slots vs the XOR swizzle
# (devlib/dev_xor.so) on C2 and energy; the 13-bit tile pattern study
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_sharded.py -k "loopback or inplace or exchange_slice" > $O/r4c_sharded.txt 2>&1 || { tail -40 $O/r4c_sharded.txt; exit 1; }
tail -8 $O/r4c_sharded.txt
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
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4c_new_$i.json 2> $O/r4c_new_$i.err || exit 1
  DTC_LIB=$D/dev_r4.so DTC_LC_TPB=-1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4c_oldlc_$i.json 2> $O/r4c_oldlc_$i.err || exit 1
  DTC_LIB=$D/dev_xor.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4c_xor_$i.json 2> $O/r4c_xor_$i.err || exit 1
  summ $O/r4c_new_$i.json $O/r4c_oldlc_$i.json $O/r4c_xor_$i.json
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --config energy --no-cpu-baseline --steps 3 --warmup 1 > $O/r4c_en_new_$i.json 2> $O/r4c_en_new_$i.err || exit 1
  DTC_LIB=$D/dev_xor.so timeout -k 10 200 python bench.py --config energy --no-cpu-baseline --steps 3 --warmup 1 > $O/r4c_en_xor_$i.json 2> $O/r4c_en_xor_$i.err || exit 1
  summ $O/r4c_en_new_$i.json $O/r4c_en_xor_$i.json
done
timeout -k 10 120 ./tools/tile13_bench > $O/r4c_tile13.txt 2>&1 || exit 1
cat $O/r4c_tile13.txt
echo ok
