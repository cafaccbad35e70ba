#!/bin/bash
# r4 session m: -m gpu with destinations off the 64-byte grid on the skew shape; cfg 5 lines
set -o pipefail
O=gpurun_out/r4m
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for op in T N; do
  timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 10 --no-cpu-baseline --no-e2e --no-extra > $O/c5$op.json 2> $O/c5$op.err || exit 1
done
for pad in 0 2 4 6 10; do
  COSTA_PROBE_LDPAD=$pad timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 10 >> $O/ldpad.txt 2>> $O/ldpad.err || exit 1
done
