#!/bin/bash
# Build the working tree's library with extra compile flags into devlib/<name>.so
# (a development A/B variant for tools/ab_libs.sh; never the product).
# Usage (container, repo root): bash tools/build_variant.sh <name> "<flags>"
set -euo pipefail
NAME=$1; FLAGS=${2:-}
P=noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd
T=$(mktemp -d)
mkdir -p devlib
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 $FLAGS"
(cd $P/csrc && { /opt/rocm/bin/hipcc $F -c dtc_kernels.hip -o $T/k.o 2>/dev/null &
                 /opt/rocm/bin/hipcc $F -c dtc_lightcone.hip -o $T/l.o 2>/dev/null &
                 /opt/rocm/bin/hipcc $F -c dtc_tile13.hip -o $T/t.o 2>/dev/null &
                 /opt/rocm/bin/hipcc $F -c dtc_engine.cpp -o $T/e.o; wait; })
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $T/k.o $T/l.o $T/t.o $T/e.o -o devlib/$NAME.so
rm -rf $T
echo devlib/$NAME.so
