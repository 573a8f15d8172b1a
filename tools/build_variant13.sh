#!/bin/bash
# Development A/B variant of the 13-site passes only (dtc_tile13.hip with extra
# flags, linked with the product's other objects from build/obj) into
# devlib/<name>.so; never the product.
# Usage (container, repo root, after make): bash tools/build_variant13.sh <name> "<flags>"
set -euo pipefail
NAME=$1; FLAGS=${2:-}
P=noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd
T=$(mktemp -d)
mkdir -p devlib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $FLAGS -c $P/csrc/dtc_tile13.hip -o $T/t.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared build/obj/dtc_kernels.o build/obj/dtc_lightcone.o $T/t.o build/obj/dtc_engine.o -o devlib/$NAME.so
rm -rf $T
echo devlib/$NAME.so
