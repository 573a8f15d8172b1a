#!/bin/bash
# r3zx: product build with the scheduler's register trackers: GPU suite,
# smoke, default bench line and its kernel-trace summary.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3zx_tests.txt 2>&1 || { tail -20 gpurun_out/r3zx_tests.txt; exit 1; }
tail -2 gpurun_out/r3zx_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r3zx_smoke.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r3zx_bench.json 2> gpurun_out/r3zx_bench.err || exit 1
cat gpurun_out/r3zx_bench.json
export TMPDIR=/tmp; R=$(pwd)
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r3zx_prof -o kt -- python $R/bench.py --no-cpu-baseline > $R/gpurun_out/r3zx_prof.json 2>/dev/null || exit 1
