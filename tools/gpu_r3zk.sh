set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/measure_configs.sh r3zk c3 c4 energy ctrl c5 > gpurun_out/r3zk_configs.txt 2>&1 || exit 1
BENCH_ARGS="--config c3" SUFFIX=_pmc_c3 bash tools/pmc_traffic.sh r3zk 1024 > gpurun_out/r3zk_pmc_c3.log 2>&1 || exit 1
BENCH_ARGS="--config energy" SUFFIX=_pmc_energy bash tools/pmc_traffic.sh r3zk 256 > gpurun_out/r3zk_pmc_energy.log 2>&1
