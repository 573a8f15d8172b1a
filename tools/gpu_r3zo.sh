set -o pipefail
cd $GRAFT_REPO_ROOT
BENCH_ARGS="--config energy" SUFFIX=_pmc_energy bash tools/pmc_traffic.sh r3zo 1024 > gpurun_out/r3zo_pmc_energy.log 2>&1 || exit 1
cp gpurun_out/r3zo_pmc_energy.json profiles/r3zo_pmc_energy.json
timeout -k 10 300 python bench.py --config energy > gpurun_out/r3zo_energy_bench.json 2> gpurun_out/r3zo_energy_bench.err
