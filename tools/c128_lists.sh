#!/bin/bash
# c128 'T' alpha, beta (cfg 4's op) at 16384^2 with 128^2 blocks: local list, and pack / unpack
# lists through the loopback exchange in one round (kernels alone) and four
set -o pipefail
O=gpurun_out/${1:-c128}; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 120 python3 tools/order_probe.py c128 16384 128 1 10 2>/dev/null | sed "s/^/local /" >> $O/c128.txt || exit 1
  for r in 1 4; do
    COSTA_LOOPBACK=1 COSTA_EXCHANGE_ROUNDS=$r timeout -k 10 120 python3 tools/order_probe.py c128 16384 128 1 10 2>/dev/null | grep "^c128" | sed "s/^/loopback rounds=$r /" >> $O/c128.txt || exit 1
  done
done
