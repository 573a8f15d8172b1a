set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3zt_gputest.txt 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3zt_smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r3zt_bench.json 2> gpurun_out/r3zt_bench.err
