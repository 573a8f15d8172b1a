# r4r: load/store register layout per nibble set (DTC_IO1_NIBS) re-measured on the
# current kernels: C2 under rocprof per library, base first and last
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_libs.sh r4r base devlib/libio40.so devlib/libioc0.so devlib/libio00.so base
