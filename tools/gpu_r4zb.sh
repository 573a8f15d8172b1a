# r4zb: recomputed echo start (dtc_kdk_redual: the forward K-D-K reruns the echo chain's first
# pass on its stored tile, one tile at three workgroups per CU) vs the two-tile dual pass;
# parity first (dual tests on the DEV library with DTC_REDUAL=192), then C2 interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
DTC_LIB=$R/devlib/libred.so DTC_REDUAL=192 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 200 --timeout-method thread -k "dual or light_cone" > gpurun_out/r4zb_tests.txt 2>&1 || { tail -20 gpurun_out/r4zb_tests.txt; exit 1; }
tail -2 gpurun_out/r4zb_tests.txt
D="DTC_LIB=$R/devlib/libred.so"
bash tools/ab_env.sh r4zb "$D DTC_REDUAL=0" "$D DTC_REDUAL=128" "$D DTC_REDUAL=64" "$D DTC_REDUAL=0" "$D DTC_REDUAL=128"
for i in 1 2 3 4 5; do python - gpurun_out/ab_r4zb_$i <<'PY'
import sys, pandas as pd
k = pd.read_csv(sys.argv[1] + "/kt_kernel_stats.csv")
k = k[k.Name.str.contains("dual")]
print(sys.argv[1], " ".join(f"{r.Name.split('(')[0].split('::')[-1]}={r.AverageNs / 1e6:.3f}" for r in k.itertuples()))
PY
done
