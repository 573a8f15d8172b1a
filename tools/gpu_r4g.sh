# r4g: the light-cone pass's PMC excess (r4e: dtc_lcw2_final FETCH_SIZE x2 = 1.44 x its
# algorithmic bytes): read-only microbenchmark of its load pattern (64-B runs) against
# 128-B / 256-B runs and contiguous tiles, timed and under a FETCH_SIZE pass; then the
# SQ counters of the C2 pass kernels at HEAD (tools/pmc_sq.sh); same-box A/B of
# dtc_lcw2_final with ordinary instead of nontemporal tile loads (devlib/lcw2_t.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 120 ./tools/run64_bench > $O/r4g_run64.txt 2>&1 || { cat $O/r4g_run64.txt; exit 1; }
cat $O/r4g_run64.txt
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_r4g_run64 -o fetch -- $R/tools/run64_bench > $R/$O/pmc_r4g_run64.log 2>&1) || { echo "fetch pass failed"; tail -5 $O/pmc_r4g_run64.log; exit 1; }
python - <<'PY'
import glob, pandas as pd
f = glob.glob("gpurun_out/pmc_r4g_run64/**/fetch_counter_collection.csv", recursive=True)[0]
d = pd.read_csv(f)
g = d.groupby("Kernel_Name").Counter_Value.mean() * 1024 / (16 * 2**30)
g.index = [n[:60] for n in g.index]
print("FETCH_SIZE per launch / 16 GiB read:")
print(g.to_string())
PY
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
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4g_nt_$i.json 2> $O/r4g_nt_$i.err || exit 1
  DTC_LIB=$R/devlib/lcw2_t.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 --warmup 1 > $O/r4g_t_$i.json 2> $O/r4g_t_$i.err || exit 1
  summ $O/r4g_nt_$i.json $O/r4g_t_$i.json
done
(cd /tmp && DTC_LIB=$R/devlib/lcw2_t.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_r4g_lct -o fetch -- python $R/bench.py --steps 1 --warmup 0 --strong-total 0 --batch 1024 --no-cpu-baseline > $R/$O/pmc_r4g_lct.log 2>&1) || { echo "lcw2_t fetch failed"; exit 1; }
python - <<'PY'
import glob, pandas as pd
f = glob.glob("gpurun_out/pmc_r4g_lct/**/fetch_counter_collection.csv", recursive=True)[0]
d = pd.read_csv(f)
d = d[d.Kernel_Name.str.contains("lcw2")]
print("lcw2 with ordinary loads: FETCH_SIZE x2 / algorithmic:", d.Counter_Value.mean() * 1024 * 2 / (16 * 2**30))
PY
bash tools/pmc_sq.sh r4g || exit 1
python tools/sq_table.py gpurun_out/pmc_r4g > $O/r4g_sq_table.md || exit 1
cat $O/r4g_sq_table.md
echo ok
