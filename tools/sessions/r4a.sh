#!/bin/bash
# r4 session a: chunked wavefront transposes (parity, cfg 5 'T' A/B) and cfg 4 orders / shapes
set -o pipefail
O=gpurun_out/r4a
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_tiles.py tests/test_gpu_cfg5.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
python3 tools/ab_bench.py $O/c5T 2 'chunk1:COSTA_TUNING=1,COSTA_TINY_CHUNK=1' 'chunk0:COSTA_TUNING=1,COSTA_TINY_CHUNK=0' -- --workload cfg5 --cfg5-op T --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
python3 tools/ab_bench.py $O/c4 1 'def:' 'ls0:COSTA_TUNING=1,COSTA_LARGE_SORT=0' 'ls2:COSTA_TUNING=1,COSTA_LARGE_SORT=2' 'sq:COSTA_TUNING=1,COSTA_FORCE_SQ=1' -- --workload cfg4 --edge 32768 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
python3 tools/ab_bench.py $O/c4b0 1 'beta0:' -- --workload cfg4 --edge 32768 --cfg4-beta0 --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 200 tools/pcie_probe 2048 > $O/pcie.log 2>&1 || exit 1
