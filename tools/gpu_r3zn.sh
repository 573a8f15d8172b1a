set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3zn_gputest.txt 2>&1 || exit 1
for b in 256 1024 256 1024; do
timeout -k 10 200 python bench.py --config energy --batch $b --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r3zn_energy_b${b}_$RANDOM.json 2>/dev/null || exit 1
done
