#!/bin/bash
# r4 session g: full -m gpu suite + smoke on the current library, then c128 transposes
set -o pipefail
O=gpurun_out/r4g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
for a in "c128 16384 128 1.0" "c128 16384 256 1.0" "c128 16384 64 1.0" "c128 16384 80 1.0" "c128 16384 128 0.0" "c128 32768 128 1.0"; do
  timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/c128.txt 2>> $O/c128.err || exit 1
done
timeout -k 10 300 python3 bench.py --workload cfg4 --edge 32768 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/c4.json 2> $O/c4.err || exit 1
