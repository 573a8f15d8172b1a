set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/measure_configs.sh r3x c3 c4 energy ctrl c5 > gpurun_out/r3x_configs.txt 2>&1 && \
bash tools/strong_projection.sh r3x > gpurun_out/r3x_strong.txt 2>&1
