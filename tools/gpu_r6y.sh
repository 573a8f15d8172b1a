set -o pipefail
mkdir -p gpurun_out
for lib in add merge addmerge; do
  DTC_LIB=$PWD/devlib/$lib.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "lcw3 or light_cone" > gpurun_out/r6y_par_$lib.txt 2>&1 || { tail -20 gpurun_out/r6y_par_$lib.txt; exit 1; }
  tail -1 gpurun_out/r6y_par_$lib.txt
done
bash tools/gpu_run.sh r6y ablibs:base,devlib/add.so,devlib/merge.so,devlib/addmerge.so,base,devlib/add.so,devlib/merge.so,devlib/addmerge.so
