#!/bin/bash
# GPU box: GPU tests, then 16384^2 'T' over element types and block sizes (tools/order_probe.py),
# cfg 2 and cfg 4 benches
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sq_check}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
: > "$OUT/blocks.log"
for cfg in "f64 16384 64 0" "c64 16384 64 0" "c128 16384 64 0" "c128 16384 80 0" "c128 16384 96 0" "c128 16384 128 1.5" \
           "c128 16384 128 0" "c128 16384 256 0" "f64 16384 256 0"; do
  timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null >> "$OUT/blocks.log" || exit 1
done
cat "$OUT/blocks.log"
bash tools/ab_bench.sh "$OUT/ab" "c2||--steps 20 --warmup 3" "c4||--workload cfg4 --steps 10 --warmup 2"
