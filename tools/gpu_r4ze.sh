# r4ze: C3's 8-site K-D-K (device kinds) at three workgroups per CU (DTC_KDK_SPLIT 49344 vs 49280), DEV library
set -o pipefail
cd $GRAFT_REPO_ROOT
R=$GRAFT_REPO_ROOT
D="DTC_LIB=$R/devlib/libdev.so"
bash tools/ab_env_c3.sh r4ze "$D DTC_KDK_SPLIT=49280" "$D DTC_KDK_SPLIT=49344" "$D DTC_KDK_SPLIT=49280" "$D DTC_KDK_SPLIT=49344"
