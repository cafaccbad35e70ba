#!/bin/bash
# r6 session s: transposes into group-writable destinations kept on the wavefront path (grouped)
# instead of the skew kernel (gpuvar/prev = the previous engine.cpp): cfg 5 'T' steps alternating,
# rocprofv3; then the GPU tests of lists, groups, skew and parity
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
export TMPDIR=/tmp
G=$GRAFT_REPO_ROOT/gpuvar
B="--steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra --workload cfg5"
timeout -k 10 600 python3 tools/ab_bench.py $O/T 3 "new:" "prev:COSTA_LIB=$G/prev/lib/libcosta_amd.so" -- $B --cfg5-op T > $O/T.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_T -o trace --output-format csv -- python3 bench.py $B --cfg5-op T > $O/prof_T.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
