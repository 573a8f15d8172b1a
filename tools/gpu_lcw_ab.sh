set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "light_cone or random_state or matches_oracle" > gpurun_out/r3t_lcw_tests.txt 2>&1 && \
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3t_lcw_on_$i.json 2> gpurun_out/r3t_lcw_on_$i.err && \
DTC_NO_LCW=1 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3t_lcw_off_$i.json 2> gpurun_out/r3t_lcw_off_$i.err || exit 1
done
