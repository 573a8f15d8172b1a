#!/bin/bash
# Round-5 development A/B (r5q/r5r, not the product): C4 (L=28) under rocprofv3
# kernel trace for library / DTC_OCTET_BITS pairs ("lib:ob", DEV builds in
# devlib/), then C5 once per library.  Usage: bash tools/r5q_c4_octet.sh <tag> lib:ob ...
set -o pipefail
TAG=$1; shift
R=$(pwd); O=$R/gpurun_out; mkdir -p $O; export TMPDIR=/tmp
cd /tmp
for spec in "$@"; do
  lib=${spec%%:*}; ob=${spec##*:}; n=${TAG}_$(basename $lib .so)_ob$ob
  DTC_LIB=$R/devlib/$lib DTC_OCTET_BITS=$ob timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$n -o kt -- python $R/bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo "$spec failed"; tail -5 $O/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$n.json')); print('$spec', round(d['value'], 2), d['ms_per_step'])"
done
