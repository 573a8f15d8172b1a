set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 ./tools/pass_pattern_bench > gpurun_out/r3u_pattern_swizzle.txt 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_energy -o run -- python bench.py --config energy --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3u_energy.json 2> gpurun_out/r3u_energy.err
