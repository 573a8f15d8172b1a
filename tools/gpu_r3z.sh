set -o pipefail
cd $GRAFT_REPO_ROOT
export DTC_LIB=$GRAFT_REPO_ROOT/devlib/libdtc_timing.so
for m in probe zsite energy; do
  echo "== $m" >> gpurun_out/r3z_phase_timing.txt
  timeout -k 10 120 python tools/phase_timing.py 256 4 $m >> gpurun_out/r3z_phase_timing.txt 2>&1 || exit 1
done
