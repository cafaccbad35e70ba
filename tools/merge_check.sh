#!/bin/bash
# -m gpu suite, then small-block transposes with and without merging (COSTA_MERGE), cfg 2 bench
set -o pipefail
O=gpurun_out/${1:-mergecheck}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for m in 1 0; do
  for cfg in "f32 16384 16 0" "f32 16384 24 0" "f32 16384 24 1" "f64 16384 24 0" "f64 16384 24 1" "c64 16384 24 0" "c128 16384 16 0" "f64 16384 256 0"; do
    COSTA_MERGE=$m timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | sed "s/^/merge=$m /" >> $O/small.txt || exit 1
  done
done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-extra > $O/bench.json 2> $O/bench.err || exit 1
bash tools/merge_loopback.sh $(basename $O)_lb || exit 1
