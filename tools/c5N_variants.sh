#!/bin/bash
# GPU box (tuning, not product): cfg 5 'N' (the wavefront path's copy list) with the
# default library against the variants under build/variants/ (tools/tiny_variants.sh), two rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-c5T_variants}
mkdir -p "$OUT"
for rep in 1 2; do
  specs=("default_$rep||--workload cfg5 --cfg5-op N --steps 20 --warmup 3")
  for d in build/variants/*/; do
    n=$(basename "$d")
    specs+=("${n}_$rep|COSTA_LIB=${d}libcosta_amd.so|--workload cfg5 --cfg5-op N --steps 20 --warmup 3")
  done
  bash tools/ab_bench.sh "$OUT" "${specs[@]}" || exit $?
done
