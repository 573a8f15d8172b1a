# r4q: device-noise dual pass (dtc_kd_dual) -- device parity tests, then a
# same-box C3 A/B against the unfused schedule (DTC_NO_DUAL), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_device.py -m gpu -v --timeout 300 --timeout-method thread > $O/r4q_tests.txt 2>&1 || { tail -30 $O/r4q_tests.txt; exit 1; }
tail -3 $O/r4q_tests.txt
for rep in 1 2; do
  for v in dual nodual; do
    if [ $v = nodual ]; then E="DTC_NO_DUAL=1"; else E="DTC_DUMMY=1"; fi
    env $E timeout -k 10 300 python -u bench.py --config c3 --no-cpu-baseline > $O/r4q_c3_${v}_$rep.json 2> $O/r4q_c3_${v}_$rep.err || { tail -5 $O/r4q_c3_${v}_$rep.err; exit 1; }
    python -c "import json; d=json.load(open('$O/r4q_c3_${v}_$rep.json')); print('$v', $rep, round(d['value'], 1), d['ms_per_step'], d['roofline']['achieved'])"
  done
done
