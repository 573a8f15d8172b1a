set -o pipefail
bash tools/gpu_run.sh r6z tests smoke || exit 1
BENCH_ARGS="--config c3" bash tools/gpu_run.sh r6z_c3 ablibs:base,devlib/add.so,base,devlib/add.so
