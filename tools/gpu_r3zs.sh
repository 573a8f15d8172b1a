set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "light_cone or matches_oracle" > gpurun_out/r3zs_tests.txt 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zs_c2_sw_$i.json 2>/dev/null && \
DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_hip_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zs_c2_base_$i.json 2>/dev/null || exit 1
done
bash tools/pmc_sq.sh r3zs > gpurun_out/r3zs_sq.log 2>&1
