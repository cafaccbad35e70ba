#!/bin/bash
# transposing wavefront pieces cut with COSTA_TR_SIDE (the side along f) on pack / unpack lists of
# small blocks through the loopback exchange (one round: kernels alone), twice
set -o pipefail
O=gpurun_out/${1:-sidelb}; mkdir -p $O
for rep in 1 2; do
  for cfg in "f64 16384 24 1" "c128 16384 16 0" "c64 16384 24 0"; do
    for side in 0 16 11 8; do
      e=""; [ $side != 0 ] && e="COSTA_TR_SIDE=$side"
      env $e COSTA_LOOPBACK=1 COSTA_EXCHANGE_ROUNDS=1 timeout -k 10 120 python3 tools/order_probe.py $cfg 10 2>/dev/null | grep "^[fc]" | sed "s/^/side=$side /" >> $O/side.txt || exit 1
    done
  done
done
