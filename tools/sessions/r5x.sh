#!/bin/bash
# r5 session x: driver-style check of the tree with the r5 copy shapes -- the -m gpu suite, smoke, and the default
# bench line (N = 1: headline, end-to-end legs, cfg 3 / 4 / 5 single-GPU slices each beside the
# reference's CPU rate).  (SKIP_TESTS=1: the bench only)
set -o pipefail
O=gpurun_out/r5x
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
fi
t0=$(date +%s.%N)
timeout -k 10 480 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
python3 -c "import sys,time; print('bench wall %.1f s' % (time.time() - float(sys.argv[1])))" $t0 > $O/bench_wall.txt
