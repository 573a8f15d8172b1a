#!/bin/bash
# Build the product library of a git revision into devlib/<name>.so (a baseline
# for tools/ab_libs.sh A/Bs against the working tree's build; never the product).
# Usage (container, repo root): bash tools/build_devlib.sh <rev> <name>
set -euo pipefail
REV=$1; NAME=$2
P=noise-resilience-in-discrete-time-crystal-realizations-on-quantum-computers_amd
T=$(mktemp -d)
mkdir -p $T/a/csrc $T/include devlib
for f in dtc_device.h dtc_kernels.h dtc_kernels.hip dtc_lightcone.hip dtc_engine.cpp dtc_rng.h; do
  git show $REV:$P/csrc/$f > $T/a/csrc/$f
done
git show $REV:include/dtc.h > $T/include/dtc.h
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17"
(cd $T/a/csrc && { /opt/rocm/bin/hipcc $F -c dtc_kernels.hip -o $T/k.o 2>/dev/null &
                   /opt/rocm/bin/hipcc $F -c dtc_lightcone.hip -o $T/l.o 2>/dev/null &
                 /opt/rocm/bin/hipcc $F -c dtc_tile13.hip -o $T/t.o 2>/dev/null &
                   /opt/rocm/bin/hipcc $F -c dtc_engine.cpp -o $T/e.o; wait; })
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared $T/k.o $T/l.o $T/t.o $T/e.o -o devlib/$NAME.so
rm -rf $T
echo devlib/$NAME.so
