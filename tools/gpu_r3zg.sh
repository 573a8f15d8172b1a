set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3zg_gputest.txt 2>&1 || exit 1
for i in 1 2; do
for c in energy ctrl; do
timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zg_${c}_new_$i.json 2>/dev/null && \
DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_hip_r3v.so timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zg_${c}_old_$i.json 2>/dev/null || exit 1
done
done
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zg_c2.json 2>/dev/null
