# round 4 first call: GPU suite + smoke + the default C2 line at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4a_gputest.txt 2>&1 || { tail -30 gpurun_out/r4a_gputest.txt; exit 1; }
tail -3 gpurun_out/r4a_gputest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4a_smoke.txt 2>&1 || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err || exit 1
cat gpurun_out/r4a_bench.json
