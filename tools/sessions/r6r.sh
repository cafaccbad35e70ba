#!/bin/bash
# r6 session r: the wavefront pieces as workgroups at the end of the group launch (default) against
# a tiny_kernel launch of their own (COSTA_FUSE_PIECES=0): cfg 5 'N' / 'T' whole steps,
# alternating fresh processes; rocprofv3 of both; then the whole -m gpu suite
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp
B="--steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra --workload cfg5"
timeout -k 10 600 python3 tools/ab_bench.py $O/N 3 "fused:" "own:COSTA_TUNING=1,COSTA_FUSE_PIECES=0" -- $B --cfg5-op N > $O/N.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/ab_bench.py $O/T 3 "fused:" "own:COSTA_TUNING=1,COSTA_FUSE_PIECES=0" -- $B --cfg5-op T > $O/T.log 2>&1 || exit 1
for op in N T; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$op -o trace --output-format csv -- python3 bench.py $B --cfg5-op $op > $O/prof_$op.log 2>&1 || exit 1
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
