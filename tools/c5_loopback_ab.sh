#!/bin/bash
# -m gpu suite, then cfg 5 through the loopback exchange (pack / unpack lists) under two
# environments, alternating, twice:  tools/c5_loopback_ab.sh TAG "ENV_A" "ENV_B"
set -o pipefail
O=gpurun_out/$1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for rep in 1 2; do for e in "$2" "$3"; do for op in N T; do
  env $e COSTA_LOOPBACK=1 timeout -k 10 300 python3 tools/c5_sort_probe.py $op 10 2>&1 | grep "^sort" | sed "s/^/[$e] /" >> $O/loopback.txt || exit 1
done; done; done
