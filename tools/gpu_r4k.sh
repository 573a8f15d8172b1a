# r4k: the 12-site light-cone end (dtc_lcw3_final) -- parity first, then a
# same-box A/B against the 10-site ends (DTC_NO_LCW3), kernel stats of both
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "lcw3 or light_cone or lcw2 or dual or matches_oracle" > $O/r4k_tests.txt 2>&1 || { tail -40 $O/r4k_tests.txt; exit 1; }
tail -2 $O/r4k_tests.txt
summ() {
python - "$@" <<'PY'
import json, sys
for f in sys.argv[1:]:
    d = json.load(open(f))
    k = d.get("kernels", {})
    print(f.split("/")[-1], round(d["value"]), {n: (round(v.get("avg_ms"), 4) if isinstance(v, dict) and v.get("avg_ms") else v.get("launches") if isinstance(v, dict) else None) for n, v in k.items()})
PY
}
for i in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4k_w3_$i.json 2> $O/r4k_w3_$i.err || exit 1
  DTC_NO_LCW3=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4k_w2_$i.json 2> $O/r4k_w2_$i.err || exit 1
  summ $O/r4k_w3_$i.json $O/r4k_w2_$i.json
done
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r4k -o kt -- python $R/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $R/$O/prof_r4k.log 2>&1) || exit 1
python - <<'PY'
import glob, pandas as pd
f = glob.glob("gpurun_out/prof_r4k/**/kt_kernel_stats.csv", recursive=True)[0]
k = pd.read_csv(f)
k["Name"] = k.Name.str.slice(0, 50)
print(k[["Name", "Calls", "AverageNs", "Percentage"]].head(12).to_string())
PY
echo ok
