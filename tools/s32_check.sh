#!/bin/bash
# GPU box: GPU tests, then 16384^2 'T' with 32^2 (and neighbouring) blocks over element types
# (tools/order_probe.py), cfg 2 and cfg 5 'T' benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-s32_check}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
: > "$OUT/blocks.log"
for cfg in "f32 16384 32 0" "f64 16384 32 0" "c64 16384 32 0" "c128 16384 32 0" "f32 16384 32 1.5" "f64 16384 32 1.5" \
           "f64 16384 24 0" "f64 16384 48 0" "f32 16384 64 0"; do
  timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null >> "$OUT/blocks.log" || exit 1
done
cat "$OUT/blocks.log"
bash tools/ab_bench.sh "$OUT/ab" "c2||--steps 20 --warmup 3" "c5T||--workload cfg5 --cfg5-op T --steps 20 --warmup 3"
