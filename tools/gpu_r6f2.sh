set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_device.py tests/test_gpu_large.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lcw3 or light_cone or device or large or l28 or site" > gpurun_out/r6f2_par_base.txt 2>&1 || { tail -20 gpurun_out/r6f2_par_base.txt; exit 1; }
tail -1 gpurun_out/r6f2_par_base.txt
DTC_LIB=$PWD/devlib/reclds.so timeout -k 10 400 python -u -m pytest tests/test_gpu_energy.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6f2_par_reclds.txt 2>&1 || { tail -20 gpurun_out/r6f2_par_reclds.txt; exit 1; }
tail -1 gpurun_out/r6f2_par_reclds.txt
bash tools/gpu_run.sh r6f2 ablibs:base,devlib/lchead.so,base,devlib/lchead.so || exit 1
BENCH_ARGS="--config c3" bash tools/gpu_run.sh r6f2_c3 ablibs:base,devlib/lchead.so,base,devlib/lchead.so || exit 1
BENCH_ARGS="--config energy" bash tools/gpu_run.sh r6f2_en ablibs:base,devlib/lchead.so,devlib/reclds.so,base,devlib/lchead.so,devlib/reclds.so || exit 1
BENCH_ARGS="--config c4" bash tools/gpu_run.sh r6f2_c4 ablibs:base,devlib/lchead.so,base,devlib/lchead.so
