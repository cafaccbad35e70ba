#!/bin/bash
# r6 session b: copies into destinations off the 64-byte grid cut at the granules (engine.cpp
# granule_split, COSTA_COPY_GRANULE=1 under COSTA_TUNING) -- parity tests with and without it,
# then tools/copy_pad_probe.py alternating; the int32 destination-block groups; where
# cfg 5's plan-cache miss spends its time (COSTA_PLAN_TRACE)
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_cblock.py tests/test_gpu_parity.py -k "cblock or unaligned_copy" > $O/pytest_default.txt 2>&1 || exit 1
COSTA_TUNING=1 COSTA_COPY_GRANULE=1 timeout -k 10 300 $T tests/test_gpu_parity.py -k "unaligned_copy or unaligned_skew or merged_small" > $O/pytest_granule.txt 2>&1 || exit 1
for r in 0 1; do
  timeout -k 10 300 python3 tools/copy_pad_probe.py 10 > $O/pad_default_$r.txt 2>&1 || exit 1
  COSTA_TUNING=1 COSTA_COPY_GRANULE=1 timeout -k 10 300 python3 tools/copy_pad_probe.py 10 > $O/pad_granule_$r.txt 2>&1 || exit 1
done
for op in N T; do
  COSTA_PLAN_TRACE=1 timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/trace_$op.json 2> $O/trace_$op.err || exit 1
done
# the headline's two unprobed pattern candidates beside kind 5, per buffer pair
timeout -k 10 300 python3 tools/pattern_probe.py 8 r6 > $O/pattern_r6.txt 2>&1 || exit 1
