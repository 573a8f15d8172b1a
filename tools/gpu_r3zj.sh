set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zj_c2_cur_$i.json 2>/dev/null && \
DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_hip_r3v.so timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zj_c2_r3v_$i.json 2>/dev/null || exit 1
done
