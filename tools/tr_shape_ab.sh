#!/bin/bash
# GPU box (tuning, not product): complex transposes (tools/order_probe.py, 16384^2, 128^2 / 256^2
# blocks, beta 0 and 1.5) and BASELINE cfg 4's single-GPU slice, default library against the
# variants under build/variants/ (tools/tiny_variants.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-tr_shape_ab}
mkdir -p "$OUT"
for lib in default build/variants/*/; do
  n=$(basename "$lib")
  [ "$lib" = default ] && L="" || L="COSTA_LIB=${lib}libcosta_amd.so"
  for cfg in "c64 16384 128 0" "c64 16384 256 1.5" "c128 16384 128 0" "c128 16384 128 1.5" "c128 16384 256 0" "f32 16384 128 0" "f32 16384 256 1.5"; do
    env $L timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | sed "s/^/$n /" >> "$OUT/probe.log"
    rc=${PIPESTATUS[0]}; [ $rc -eq 0 ] || { echo "rc=$rc $n $cfg"; exit 1; }
  done
done
cat "$OUT/probe.log"
specs=("c4_default||--workload cfg4 --steps 10 --warmup 2")
for d in build/variants/*/; do
  n=$(basename "$d")
  specs+=("c4_${n}|COSTA_LIB=${d}libcosta_amd.so|--workload cfg4 --steps 10 --warmup 2")
done
specs+=("c4_default_b||--workload cfg4 --steps 10 --warmup 2")
bash tools/ab_bench.sh "$OUT/ab" "${specs[@]}"
