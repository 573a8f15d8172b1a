set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "light_cone or matches_oracle" > gpurun_out/r3zp_tests.txt 2>&1 || exit 1
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zp_c2_spec_$i.json 2>/dev/null && \
DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_hip_base.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zp_c2_base_$i.json 2>/dev/null || exit 1
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r3zp -o kt -- python $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --steps 2 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_r3zp.log 2>&1
