#!/bin/bash
# GPU box: GPU tests, then fp64 16384^2 'T' over block sizes (tools/order_probe.py) and cfg 2's bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-sq_check}
mkdir -p "$OUT"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -2 "$OUT/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
: > "$OUT/blocks.log"
for rep in 1 2; do
  for cfg in "f64 16384 64 0" "f64 16384 64 1.5" "f64 16384 32 0" "f64 16384 48 0" "f64 16384 96 0" "f64 16384 128 0" "f64 16384 256 0"; do
    timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null >> "$OUT/blocks.log" || exit 1
  done
done
sort "$OUT/blocks.log"
bash tools/ab_bench.sh "$OUT/ab" "c2||--steps 20 --warmup 3"
