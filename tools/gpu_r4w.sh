# r4w: SQ counters of the energy line's pass kernels (B=64), one rocprofv3 --pmc pass per set
set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--config energy" bash tools/pmc_sq.sh r4w_energy && python tools/sq_table.py gpurun_out/pmc_r4w_energy kdk kick > gpurun_out/r4w_energy_sq.md && cat gpurun_out/r4w_energy_sq.md
