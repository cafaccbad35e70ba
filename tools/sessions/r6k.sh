#!/bin/bash
# r6 session k: destination-block groups built on the GPU (device_lists.hip) -- host == GPU work
# lists (test_gpu_work_lists.py), the cfg 5 / group / device-planner tests on the default builder,
# and the plan-cache miss traced (COSTA_PLAN_TRACE) on the cfg 5 lines
set -o pipefail
O=gpurun_out/r6k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_work_lists.py > $O/pytest_wl.txt 2>&1 || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cblock.py tests/test_gpu_cfg5.py tests/test_gpu_device_plan.py > $O/pytest_c5.txt 2>&1 || exit 1
for op in N T; do
  COSTA_PLAN_TRACE=1 timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op $op --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/trace_$op.json 2> $O/trace_$op.err || exit 1
done
