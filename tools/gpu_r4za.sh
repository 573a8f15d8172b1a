# r4za: the 12-site light-cone end at three / two workgroups per CU (more VGPRs, fewer waves)
# vs the product's four, C2 interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_libs.sh r4za base devlib/liblcw3_w3.so devlib/liblcw3_w2.so base devlib/liblcw3_w3.so
for i in 1 2 3 4 5; do python - gpurun_out/ab_r4za_$i <<'PY'
import sys, pandas as pd
k = pd.read_csv(sys.argv[1] + "/kt_kernel_stats.csv")
k = k[k.Name.str.contains("lcw3")]
print(sys.argv[1], " ".join(f"{r.Name.split('(')[0].split('::')[-1]}={r.AverageNs / 1e6:.3f}" for r in k.itertuples()))
PY
done
