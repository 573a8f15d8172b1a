set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_device.py tests/test_gpu_parity.py -k "device or matches_oracle or random_state" > gpurun_out/r3y_device_tests.txt 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3y_c3_new_$i.json 2> gpurun_out/r3y_c3_new_$i.err && \
DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_hip_r3v.so timeout -k 10 200 python bench.py --config c3 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3y_c3_old_$i.json 2> gpurun_out/r3y_c3_old_$i.err || exit 1
done
