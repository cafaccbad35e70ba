#!/bin/bash
# r4 session q: the 128 KiB destination panels as shipped (default) against none (-1)
set -o pipefail
O=gpurun_out/r4q
mkdir -p $O
for r in 1 2; do
for a in "c128 32768 128 1.0" "f64 32768 128 1.0" "c64 32768 128 1.0" "f32 32768 256 0.0" "f64 16384 256 0.0"; do
  for h in 0 -1; do
    echo -n "H=$h " >> $O/panels.txt
    COSTA_TUNING=1 COSTA_PANEL_ROWS=$h timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/panels.txt 2>> $O/panels.err || exit 1
  done
done
done
timeout -k 10 300 python3 bench.py --workload cfg4 --edge 32768 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/c4.json 2> $O/c4.err || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
