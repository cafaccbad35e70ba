#!/bin/bash
# -m gpu suite, cfg 5 bench lines and the loopback pack / unpack times of the current library
set -o pipefail
O=gpurun_out/${1:-c5check}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for op in N T; do
  timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 10 --no-cpu-baseline --no-e2e --no-extra > $O/c5$op.json 2> $O/c5$op.err || exit 1
  COSTA_LOOPBACK=1 timeout -k 10 300 python3 tools/c5_sort_probe.py $op 10 2>&1 | grep "^sort" >> $O/loopback.txt || exit 1
done
