#!/bin/bash
# r6 session g: the group builder's phases after the gather / single-thread marking / 16-bit digits
# (COSTA_PLAN_TRACE, cfg 5 'N' / 'T' lines), the cfg 5 GPU tests on it; the reference's multi-rank
# CPU baselines bench.py runs beside an N-rank line, rehearsed on this box's host at N = 2, 4, 8
# (MPICH child processes only, no GPU: tools/mr_baseline_probe.py)
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py > $O/pytest_c5.txt 2>&1 || exit 1
for op in N T; do
  COSTA_PLAN_TRACE=1 timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/trace_$op.json 2> $O/trace_$op.err || exit 1
done
timeout -k 10 600 python3 tools/mr_baseline_probe.py 2 4 8 > $O/mr_baseline.txt 2> $O/mr_baseline.err || exit 1
