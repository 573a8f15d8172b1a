# r4zh: energy line kernel trace at HEAD (where the r4zg step's +8 ms goes)
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
O=gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_r4zh_energy -o kt -- python $R/bench.py --config energy --no-cpu-baseline > $R/$O/prof_r4zh_energy.log 2>&1) || { echo "trace failed"; tail -5 $O/prof_r4zh_energy.log; exit 1; }
tail -1 $O/prof_r4zh_energy.log
echo ok
