# r4s: the 8-site (<6>) K-D-K at three workgroups per CU (half-tile re-layouts)
# re-measured on the current kernels: DEV library, DTC_KDK_SPLIT default (49280)
# vs + bit 6 (49344), interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
bash tools/ab_env.sh r4s "DTC_LIB=$R/devlib/libdev.so DTC_KDK_SPLIT=49280" "DTC_LIB=$R/devlib/libdev.so DTC_KDK_SPLIT=49344" "DTC_LIB=$R/devlib/libdev.so DTC_KDK_SPLIT=49280" "DTC_LIB=$R/devlib/libdev.so DTC_KDK_SPLIT=49344"
