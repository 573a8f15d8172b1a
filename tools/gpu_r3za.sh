set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_energy.py > gpurun_out/r3za_energy_tests.txt 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --config energy --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3za_energy_new_$i.json 2>/dev/null && \
DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_hip_r3v.so timeout -k 10 200 python bench.py --config energy --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3za_energy_old_$i.json 2>/dev/null || exit 1
done
DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_timing.so timeout -k 10 120 python tools/phase_timing.py 256 4 energy > gpurun_out/r3za_phase_energy.txt 2>&1
