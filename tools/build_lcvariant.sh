#!/bin/bash
# Development A/B variant of the light-cone translation unit only: compiles
# dtc_lightcone.hip with extra flags and links it with the product's other
# objects from build/obj (run `make` first) into devlib/<name>.so.
# Usage (container, repo root): bash tools/build_lcvariant.sh <name> "<flags>"
set -euo pipefail
NAME=$1; FLAGS=${2:-}
P=noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd
T=$(mktemp -d)
mkdir -p devlib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 $FLAGS -c $P/csrc/dtc_lightcone.hip -o $T/l.o 2>/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared build/obj/dtc_kernels.o $T/l.o build/obj/dtc_tile13.o build/obj/dtc_engine.o -o devlib/$NAME.so
rm -rf $T
echo devlib/$NAME.so
