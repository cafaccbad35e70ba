#!/bin/bash
# r4 session t: every op merged before sub-tiling (default) -- -m gpu, headline, ragged blocks
set -o pipefail
O=gpurun_out/r4t
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-extra > $O/bench.json 2> $O/bench.err || exit 1
for a in "c128 16384 80 1.0" "f64 16384 100 0.0" "f64 16384 256 0.0" "c128 16384 128 1.0" "f32 16384 96 1.0"; do
  for m in 2 1; do
    echo -n "merge=$m " >> $O/merge.txt
    COSTA_TUNING=1 COSTA_MERGE=$m timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/merge.txt 2>> $O/merge.err || exit 1
  done
done
