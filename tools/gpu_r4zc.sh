# r4zc: the measure-only final passes (dtc_*_final) at three workgroups per CU with half-tile
# re-layouts vs two (product), C3 interleaved (its echo chains end in kick-only final passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--config c3" bash tools/ab_libs.sh r4zc base devlib/libfin3.so base devlib/libfin3.so
for i in 1 2 3 4; do python - gpurun_out/ab_r4zc_$i <<'PY'
import sys, pandas as pd
k = pd.read_csv(sys.argv[1] + "/kt_kernel_stats.csv")
k = k[k.Name.str.contains("final")]
print(sys.argv[1], " ".join(f"{r.Name.split('(')[0].split('::')[-1]}={r.AverageNs / 1e6:.3f}" for r in k.itertuples()))
PY
done
