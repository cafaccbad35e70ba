#!/bin/bash
# r6 session t: single-op components grouped too (no wavefront pieces left in cfg 5; gpuvar/new)
# against the shipped build: cfg 5 'N' / 'T' steps alternating; the whole -m gpu suite on the
# new build (COSTA_LIB)
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp
G=$GRAFT_REPO_ROOT/gpuvar
B="--steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra --workload cfg5"
timeout -k 10 600 python3 tools/ab_bench.py $O/N 3 "new:COSTA_LIB=$G/new/lib/libcosta_amd.so" "prev:" -- $B --cfg5-op N > $O/N.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/ab_bench.py $O/T 3 "new:COSTA_LIB=$G/new/lib/libcosta_amd.so" "prev:" -- $B --cfg5-op T > $O/T.log 2>&1 || exit 1
COSTA_LIB=$G/new/lib/libcosta_amd.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
