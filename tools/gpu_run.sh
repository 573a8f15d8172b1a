#!/bin/bash
# One parameterised GPU-box recipe (replaces the per-call gpu_r3*/gpu_r4* scripts).
# Usage (gpurun, repo root):  bash tools/gpu_run.sh <tag> <step> [<step> ...]
# Steps run in order; the first failing step ends the call (no retries):
#   c2                 bench line + rocprof kernel stats + PMC at B=1024 (tools/measure_c2.sh)
#   bench:<cfg>        bench.py --config <cfg> line -> gpurun_out/<tag>_<cfg>_bench.json
#   trace:<cfg>        the same command under rocprofv3 --kernel-trace --stats -> prof_<tag>_<cfg>/
#   pmc:<cfg>:<B>[:L]  FETCH_SIZE / WRITE_SIZE passes at batch B -> <tag>_pmc_<cfg>.json
#                      (c2: <tag>_pmc.json, the headline line's)
#   smoke              __graft_entry__.smoke()
#   tests[:<expr>]     pytest -m gpu [-k <expr>] -> <tag>_gputest.txt
#   ab:<VAR=v>,<VAR=v> interleaved env A/B of the C2 line under rocprof (tools/ab_env.sh)
#   ablibs:<l1>,<l2>.. interleaved library A/B of the C2 line under rocprof (tools/ab_libs.sh;
#                      "base" = the product library, else a devlib/*.so built in the container)
#   stage              copy this call's PMC summaries (gpurun_out/<tag>*_pmc*.json) into
#                      profiles/ of the box's copy, so later bench steps cite them
#   exec:<file>        run gpu_bin/<file> (a probe built in the container) -> <tag>_<file>.txt
#   libtests:<lib>:<k> pytest -m gpu -k <k> against devlib/<lib>.so (a variant's parity before
#                      its A/B) -> <tag>_par_<lib>.txt
#   configs            every non-C2 line once (tools/measure_configs.sh)
set -o pipefail
TAG=$1; shift
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R=$(pwd); O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  echo "== $step"
  case $step in
    c2)
      bash tools/measure_c2.sh $TAG || exit 1 ;;
    bench:*)
      c=${step#bench:}
      timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > $O/${TAG}_${c}_bench.json 2> $O/${TAG}_${c}_bench.err || { tail -5 $O/${TAG}_${c}_bench.err; exit 1; }
      python -c "import json; d=json.load(open('$O/${TAG}_${c}_bench.json')); r=d.get('roofline') or {}; print('$c', d['value'], r.get('achieved'), r.get('traffic'))" ;;
    trace:*)
      c=${step#trace:}
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_${TAG}_$c -o kt -- python $R/bench.py --config $c --no-cpu-baseline --steps 2 --warmup 1 > $R/$O/prof_${TAG}_$c.log 2>&1) || { echo "$c trace failed"; tail -5 $O/prof_${TAG}_$c.log; exit 1; } ;;
    pmc:*)
      IFS=: read -r _ c b l <<< "$step"
      if [ "$c" = c2 ]; then  # the headline line reads <tag>_pmc.json
        L=${l:-20} BENCH_ARGS="" SUFFIX=_pmc bash tools/pmc_traffic.sh $TAG $b || exit 1
      else
        L=${l:-20} BENCH_ARGS="--config $c" SUFFIX=_pmc_$c bash tools/pmc_traffic.sh $TAG $b || exit 1
      fi ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/${TAG}_smoke.txt 2>&1 || { cat $O/${TAG}_smoke.txt; exit 1; }
      tail -1 $O/${TAG}_smoke.txt ;;
    tests*)
      k=${step#tests}; k=${k#:}
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${k:+-k "$k"} > $O/${TAG}_gputest.txt 2>&1; rc=$?
      tail -4 $O/${TAG}_gputest.txt
      [ $rc -eq 0 ] || exit $rc ;;
    ab:*)
      IFS=, read -ra settings <<< "${step#ab:}"
      bash tools/ab_env.sh $TAG "${settings[@]}" || exit 1 ;;
    ablibs:*)
      IFS=, read -ra libs <<< "${step#ablibs:}"
      bash tools/ab_libs.sh $TAG "${libs[@]}" || exit 1 ;;
    stage)
      cp $O/${TAG}*_pmc*.json profiles/ || exit 1
      ls profiles/${TAG}*_pmc*.json ;;
    exec:*)
      f=${step#exec:}
      timeout -k 10 300 gpu_bin/$f > $O/${TAG}_$f.txt 2>&1 || { tail -5 $O/${TAG}_$f.txt; exit 1; }
      cat $O/${TAG}_$f.txt ;;
    libtests:*)
      IFS=: read -r _ lib k <<< "$step"
      DTC_LIB=$R/devlib/$lib.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$k" > $O/${TAG}_par_$lib.txt 2>&1 || { tail -20 $O/${TAG}_par_$lib.txt; exit 1; }
      tail -1 $O/${TAG}_par_$lib.txt ;;
    configs)
      bash tools/measure_configs.sh $TAG || exit 1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "gpu_run $TAG done"
