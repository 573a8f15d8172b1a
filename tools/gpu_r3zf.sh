set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_sq.sh r3zf > gpurun_out/r3zf_sq.log 2>&1 || exit 1
BENCH_ARGS="--config c3" bash tools/pmc_sq.sh r3zf_c3 >> gpurun_out/r3zf_sq.log 2>&1
