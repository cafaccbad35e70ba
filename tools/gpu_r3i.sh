#!/bin/bash
# r3: shifted stores for unaligned destinations: parity then timings
set -o pipefail
O=gpurun_out/${1:-r3i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "unaligned or mixed or special" > $O/gputest.log 2>&1 &&
timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/sides.log 2>&1 &&
COSTA_MISDST_MODE=2 timeout -k 10 300 python3 tools/unaligned_probe.py 10 sides > $O/sides_xcd.log 2>&1 &&
timeout -k 10 300 python3 tools/unaligned_probe.py 10 > $O/blocks.log 2>&1
