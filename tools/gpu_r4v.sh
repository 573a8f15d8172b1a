# r4v: timing probe (wrong results by design): the 12-site light-cone end reading
# window-contiguous tiles (DTC_LCW3_CONTIG_TIMING) vs the product's 16-B pieces
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_libs.sh r4v base devlib/liblccontig.so base devlib/liblccontig.so
for i in 1 2 3 4; do python - gpurun_out/ab_r4v_$i <<'PY'
import sys, pandas as pd
k = pd.read_csv(sys.argv[1] + "/kt_kernel_stats.csv")
k = k[k.Name.str.contains("lc")]
print(sys.argv[1], " ".join(f"{r.Name.split('(')[0].split('::')[-1]}={r.AverageNs / 1e6:.3f}" for r in k.itertuples()))
PY
done
