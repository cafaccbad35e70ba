#!/bin/bash
# r5 session ar: the -m gpu suite and smoke once more on a fresh box (the final tree)
set -o pipefail
O=gpurun_out/r5ar
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
