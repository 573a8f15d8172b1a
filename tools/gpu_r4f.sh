# r4f: alternating layouts (each pass stores its tile contiguously in its own
# group's layout; F/E ping-pong) -- parity (new test + the dual / light-cone
# tests), the dual pass's schedule/byte probe (development library), then a
# same-box A/B of the product vs DTC_NO_ALT on C2 and C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
for a in "13 9 circular_left vacuum 0 0.1" "20 12 x vacuum 0 0.05"; do
  for m in dual no_dual; do
    f=$O/r4f_probe_$(echo $a | tr ' ' '_')_$m.txt
    DTC_LIB=$R/devlib/dev.so timeout -k 10 120 python tools/dual_sched_probe.py $a $m > $f 2>&1 || { tail -5 $f; exit 1; }
    grep "^kind" $f
  done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 300 --timeout-method thread -k "alternating or light_cone or dual or lcw2 or matches_oracle" > $O/r4f_tests.txt 2>&1; rc=$?
tail -15 $O/r4f_tests.txt
[ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || exit 1
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
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4f_alt_$i.json 2> $O/r4f_alt_$i.err || exit 1
  DTC_NO_ALT=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4f_noalt_$i.json 2> $O/r4f_noalt_$i.err || exit 1
  summ $O/r4f_alt_$i.json $O/r4f_noalt_$i.json
done
for i in 1 2; do
  timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 > $O/r4f_c3alt_$i.json 2> $O/r4f_c3alt_$i.err || exit 1
  DTC_NO_ALT=1 timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 > $O/r4f_c3noalt_$i.json 2> $O/r4f_c3noalt_$i.err || exit 1
  summ $O/r4f_c3alt_$i.json $O/r4f_c3noalt_$i.json
done
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r4f -o kt -- python $R/bench.py --no-cpu-baseline --steps 3 --warmup 1 > $R/$O/prof_r4f.log 2>&1 || exit 1
cd $R && python - <<'PY'
import glob, pandas as pd
f = glob.glob("gpurun_out/prof_r4f/**/kt_kernel_stats.csv", recursive=True)[0]
k = pd.read_csv(f)
print(k[["Name", "Calls", "AverageNs", "Percentage"]].head(12).to_string())
PY
echo ok
