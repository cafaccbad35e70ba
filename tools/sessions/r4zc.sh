#!/bin/bash
# r4 session zc: the -m gpu suite, smoke and the default bench line on the final build
set -o pipefail
O=gpurun_out/r4zc
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -x -q -m gpu > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
