set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3ze_gputest.txt 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3ze_c4_new_$i.json 2>/dev/null && \
DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_hip_r3v.so timeout -k 10 200 python bench.py --config c4 --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3ze_c4_old_$i.json 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --config c5 > gpurun_out/r3ze_c5.json 2> gpurun_out/r3ze_c5.err
