# r4o: workgroups per CU of the measurement passes (development library,
# DTC_KDK_SPLIT): energy and C4 with the 12-site (A) and/or 8-site (B)
# per-site/energy K-D-K at two instead of three workgroups per CU
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
D=$R/devlib/dev.so
summ() {
python - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    k = d.get("kernels", {})
    print(f.split("/")[-1], round(d["value"], 1), {n: (round(v.get("avg_ms"), 4) if isinstance(v, dict) and v.get("avg_ms") else None) for n, v in k.items()})
PY
}
for i in 1 2; do
  for v in 49280 16512 32896 128; do
    DTC_LIB=$D DTC_KDK_SPLIT=$v timeout -k 10 200 python bench.py --config energy --no-cpu-baseline --steps 3 --warmup 1 > $O/r4o_en_${v}_$i.json 2> $O/r4o_en_${v}_$i.err || exit 1
  done
  summ $O/r4o_en_49280_$i.json $O/r4o_en_16512_$i.json $O/r4o_en_32896_$i.json $O/r4o_en_128_$i.json
done
for v in 49280 32896; do
  DTC_LIB=$D DTC_KDK_SPLIT=$v timeout -k 10 300 python bench.py --config c4 --steps 2 --warmup 1 > $O/r4o_c4_${v}.json 2> $O/r4o_c4_${v}.err || exit 1
done
summ $O/r4o_c4_49280.json $O/r4o_c4_32896.json
echo ok
