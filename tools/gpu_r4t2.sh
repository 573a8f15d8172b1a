# r4t2: octet run length g = 7 vs 6 (DTC_OCTET_BITS, DEV library), C2 interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
D="DTC_LIB=$R/devlib/libdev.so"
bash tools/ab_env.sh r4t2 "$D DTC_OCTET_BITS=6" "$D DTC_OCTET_BITS=7" "$D DTC_OCTET_BITS=6" "$D DTC_OCTET_BITS=7"
