#!/bin/bash
# r4 session zn: the persistent transposing kernel (next item's loads issued before the current
# item's stores; tuning knob COSTA_PERSIST=1) against the shipped one
set -o pipefail
O=gpurun_out/r4zn
mkdir -p $O
COSTA_TUNING=1 COSTA_PERSIST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_parity.py -x -q > $O/pytest_persist.log 2>&1 || exit 1
for rep in 1 2 3; do
  for p in 0 1; do
    for a in "f64 16384 256 0.0 20" "f64 32768 256 0.0 10" "f32 16384 256 0.0 20" "f64 16384 128 0.0 20"; do
      echo -n "persist $p " >> $O/persist.txt
      COSTA_TUNING=1 COSTA_PERSIST=$p timeout -k 10 200 python3 tools/order_probe.py $a >> $O/persist.txt 2>> $O/err.txt || exit 1
    done
  done
done
