set -o pipefail
cd $GRAFT_REPO_ROOT
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zu_c2_default_$i.json 2>/dev/null && \
DTC_KDK_SPLIT=49344 timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zu_c2_split6_$i.json 2>/dev/null || exit 1
done
