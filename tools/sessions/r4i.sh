#!/bin/bash
# r4 session i: direct-DMA host pipeline over page-locked caller memory
set -o pipefail
O=gpurun_out/r4i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_loopback.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
COSTA_HOST_PIPE_TRACE=1 timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-extra > $O/bench.json 2> $O/bench.err || exit 1
