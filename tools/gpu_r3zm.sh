set -o pipefail
cd $GRAFT_REPO_ROOT
LW=$GRAFT_REPO_ROOT/devlib/libdtc_lastwave.so
DTC_LIB=$LW timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_energy.py tests/test_gpu_parity.py tests/test_gpu_sharded.py -k "energy or matches_oracle or sharded or virtual or zsite or apply" > gpurun_out/r3zm_tests.txt 2>&1 || exit 1
for i in 1 2; do
for c in energy c4; do
timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zm_${c}_base_$i.json 2>/dev/null && \
DTC_LIB=$LW timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zm_${c}_lw_$i.json 2>/dev/null || exit 1
done
done
