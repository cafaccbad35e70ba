#!/bin/bash
# GPU box (tuning, not product): cfg 2 with the default library and the fp64 transpose shape
# variants under build/variants/ (tools/tiny_variants.sh), interleaved, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-shape_ab}
mkdir -p "$OUT"
for rep in 1 2; do
  specs=("default_$rep||--steps 20 --warmup 3")
  for d in build/variants/*/; do
    n=$(basename "$d")
    specs+=("${n}_$rep|COSTA_LIB=${d}libcosta_amd.so|--steps 20 --warmup 3")
  done
  bash tools/ab_bench.sh "$OUT" "${specs[@]}" || exit $?
done
