# r4m: lcw3 with one row swap fewer (devlib/lcw3b.so) -- its light-cone
# parity, then a same-box A/B against the product on C2
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
DTC_LIB=$R/devlib/lcw3b.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "lcw3 or light_cone" > $O/r4m_tests.txt 2>&1 || { tail -30 $O/r4m_tests.txt; exit 1; }
tail -2 $O/r4m_tests.txt
summ() {
python - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    k = d.get("kernels", {})
    print(f.split("/")[-1], round(d["value"]), {n: (round(v.get("avg_ms"), 4) if isinstance(v, dict) and v.get("avg_ms") else None) for n, v in k.items()})
PY
}
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4m_prod_$i.json 2> $O/r4m_prod_$i.err || exit 1
  DTC_LIB=$R/devlib/lcw3b.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4m_b_$i.json 2> $O/r4m_b_$i.err || exit 1
  summ $O/r4m_prod_$i.json $O/r4m_b_$i.json
done
echo ok
