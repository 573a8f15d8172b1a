set -o pipefail
mkdir -p gpurun_out
DTC_LIB=$PWD/devlib/mc3regrec.so timeout -k 10 400 python -u -m pytest tests/test_gpu_energy.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6j_par_mc3regrec.txt 2>&1 || { tail -20 gpurun_out/r6j_par_mc3regrec.txt; exit 1; }
tail -1 gpurun_out/r6j_par_mc3regrec.txt
BENCH_ARGS="--config energy" bash tools/gpu_run.sh r6j_en ablibs:base,devlib/mc3regrec.so,base,devlib/mc3regrec.so,base,devlib/mc3regrec.so
