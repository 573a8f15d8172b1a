# r4t: octet run length 2^g amplitudes, g = 4 / 5 / 6 (DTC_OCTET_BITS, DEV library), C2 interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
D="DTC_LIB=$R/devlib/libdev.so"
bash tools/ab_env.sh r4t "$D DTC_OCTET_BITS=6" "$D DTC_OCTET_BITS=4" "$D DTC_OCTET_BITS=5" "$D DTC_OCTET_BITS=6" "$D DTC_OCTET_BITS=4"
