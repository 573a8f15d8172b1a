set -o pipefail
mkdir -p gpurun_out
DTC_LIB=$PWD/devlib/swaplate.so timeout -k 10 600 python -u -m pytest tests/test_gpu_c5_l34.py tests/test_gpu_sharded.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6h_par_swaplate.txt 2>&1 || { tail -20 gpurun_out/r6h_par_swaplate.txt; exit 1; }
tail -1 gpurun_out/r6h_par_swaplate.txt
BENCH_ARGS="--config c5" bash tools/gpu_run.sh r6h_c5 ablibs:base,devlib/swaplate.so,base,devlib/swaplate.so
