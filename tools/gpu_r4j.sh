# r4j: read patterns incl. 16-B pieces (a 12-site light-cone window without
# column bits), timed and under a FETCH_SIZE pass
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 120 ./tools/run64_bench > $O/r4j_run64.txt 2>&1 || { cat $O/r4j_run64.txt; exit 1; }
cat $O/r4j_run64.txt
export TMPDIR=/tmp
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/$O/pmc_r4j_run64 -o fetch -- $R/tools/run64_bench > $R/$O/pmc_r4j_run64.log 2>&1) || { echo "fetch pass failed"; tail -5 $O/pmc_r4j_run64.log; exit 1; }
python - <<'PY'
import glob, pandas as pd
f = glob.glob("gpurun_out/pmc_r4j_run64/**/fetch_counter_collection.csv", recursive=True)[0]
d = pd.read_csv(f)
g = d.groupby("Kernel_Name").Counter_Value.mean() * 1024 / (16 * 2**30)
g.index = [n[:40] for n in g.index]
print("FETCH_SIZE per launch / 16 GiB read:")
print(g.to_string())
PY
