#!/bin/bash
# r4 session v: copy skew cut, reworked (32 columns of loads in flight per wavefront)
set -o pipefail
O=gpurun_out/r4v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for a in "f64 16384 256 0.0" "f64 16384 128 1.0" "f32 16384 256 0.0"; do
  for pad in 2 4 8; do
    for sk in 1 0; do
      echo -n "skew=$sk " >> $O/copy_ldpad.txt
      COSTA_TUNING=1 COSTA_SKEW=$sk COSTA_PROBE_OP=N COSTA_PROBE_LDPAD=$pad timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/copy_ldpad.txt 2>> $O/err.txt || exit 1
    done
  done
done
