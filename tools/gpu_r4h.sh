# r4h: light-cone parity after the ordinary-load change, then a same-box A/B of
# the 8-site (column) passes' nontemporal hints: product (NT loads + stores),
# ntb1 (NT loads, ordinary stores), ntb2 (ordinary loads, NT stores)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "light_cone or lcw2 or dual or matches_oracle" > $O/r4h_tests.txt 2>&1 || { tail -30 $O/r4h_tests.txt; exit 1; }
tail -2 $O/r4h_tests.txt
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
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4h_prod_$i.json 2> $O/r4h_prod_$i.err || exit 1
  DTC_LIB=$R/devlib/ntb1.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4h_ntb1_$i.json 2> $O/r4h_ntb1_$i.err || exit 1
  DTC_LIB=$R/devlib/ntb2.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4h_ntb2_$i.json 2> $O/r4h_ntb2_$i.err || exit 1
  summ $O/r4h_prod_$i.json $O/r4h_ntb1_$i.json $O/r4h_ntb2_$i.json
done
export TMPDIR=/tmp
for v in prod ntb1 ntb2; do
  L=""; [ $v != prod ] && L=$R/devlib/$v.so
  (cd /tmp && DTC_LIB=${L:-$R/noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd/lib/libdtc_hip.so} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r4h_$v -o kt -- python $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/$O/prof_r4h_$v.log 2>&1) || exit 1
done
python - <<'PY'
import glob, pandas as pd
for v in ("prod", "ntb1", "ntb2"):
    f = glob.glob(f"gpurun_out/prof_r4h_{v}/**/kt_kernel_stats.csv", recursive=True)[0]
    k = pd.read_csv(f)
    k["Name"] = k.Name.str.slice(0, 48)
    print(v); print(k[["Name", "Calls", "AverageNs"]].head(6).to_string())
PY
echo ok
