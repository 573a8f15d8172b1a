# r4u: dual <7> pass with full-tile LDS re-layouts (DTC_DUAL_FULL=128: 256 VGPRs, 27 spilled) vs
# the product's half-tile ones, C2 interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab_libs.sh r4u base devlib/libdf80.so base devlib/libdf80.so
