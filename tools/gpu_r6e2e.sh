# Round-6 end-of-round measurement at HEAD (GPU box, repo root): the C2 line with its rocprof
# kernel stats and PMC traffic passes, then every other config's line.
set -o pipefail
bash tools/measure_c2.sh r6e || exit 1
bash tools/measure_configs.sh r6e c3 c4 energy ctrl c5 || exit 1
