#!/bin/bash
# r6 session p: destination-block group kernel variants (gpuvar/, tools/build_variant.sh) on cfg 5:
# 'N' chunk loads a lane in flight 6 / 12 (8 shipped), default-policy stores; 'T' 20 dword loads a
# lane (16 shipped), default-policy stores
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp
G=$GRAFT_REPO_ROOT/gpuvar
B="--steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra --workload cfg5"
timeout -k 10 600 python3 tools/ab_bench.py $O/N 3 "base:" "uv6:COSTA_LIB=$G/uv6/lib/libcosta_amd.so" "uv12:COSTA_LIB=$G/uv12/lib/libcosta_amd.so" "cbst:COSTA_LIB=$G/cbst/lib/libcosta_amd.so" -- $B --cfg5-op N > $O/N.log 2>&1 || exit 1
timeout -k 10 600 python3 tools/ab_bench.py $O/T 3 "base:" "u20:COSTA_LIB=$G/u20/lib/libcosta_amd.so" "cbst:COSTA_LIB=$G/cbst/lib/libcosta_amd.so" -- $B --cfg5-op T > $O/T.log 2>&1 || exit 1
