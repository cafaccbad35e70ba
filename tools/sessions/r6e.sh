#!/bin/bash
# r6 session e: the tree with the r6 defaults (4-byte copy groups on 16-byte chunk loads in XCD
# column bands, granule-cut copies, the radix-sorted group builder, the pack stream) -- the -m gpu
# suite, smoke, the default bench line; cfg 5 'N' / 'T' lines with the first call's host time
# (COSTA_PLAN_TRACE); the granule-cut copies in destination-address order (COSTA_LARGE_SORT=2)
set -o pipefail
O=gpurun_out/r6e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
for op in N T; do
  COSTA_PLAN_TRACE=1 timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra > $O/c5$op.json 2> $O/c5$op.err || exit 1
done
timeout -k 10 300 python3 tools/copy_pad_probe.py 10 > $O/pad_default.txt 2>&1 || exit 1
COSTA_TUNING=1 COSTA_LARGE_SORT=2 timeout -k 10 300 python3 tools/copy_pad_probe.py 10 > $O/pad_addr.txt 2>&1 || exit 1
