#!/bin/bash
# r5 session e: (1) the headline with one destination column per store instruction (COSTA_TR_STAGE
# 6, tuning build) against the shipped kernel and LDS-DMA staging (1), alternating, and its UTCL1
# counters (r5c: the transpose stalls 10x longer than the one-vector copy on the UTCL1 in-flight
# limit); (2) cfg 5 'T' / 'N' on smaller destination-block groups (tuning builds of the group
# budget and threads)
set -o pipefail
O=gpurun_out/r5e
mkdir -p $O
export TMPDIR=/tmp
V=gpuvar
timeout -k 10 400 python3 tools/ab_bench.py $O/hl 3 shipped: st1:COSTA_LIB=$V/st1/lib/libcosta_amd.so \
  st6:COSTA_LIB=$V/st6/lib/libcosta_amd.so -- --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extra"
COSTA_LIB=$V/st6/lib/libcosta_amd.so timeout -s KILL 150 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE -d $O/p4 -o p4 --output-format csv -- $B > $O/p4.log 2>&1 || exit 1
timeout -k 10 400 python3 tools/ab_bench.py $O/c5T 2 c4:COSTA_LIB=$V/cbC4/lib/libcosta_amd.so \
  c2:COSTA_LIB=$V/cbC2/lib/libcosta_amd.so c4u32:COSTA_LIB=$V/cbC4U32/lib/libcosta_amd.so \
  t128c4:COSTA_LIB=$V/cbT128C4/lib/libcosta_amd.so t128c8:COSTA_LIB=$V/cbT128C8/lib/libcosta_amd.so \
  wave:COSTA_TUNING=1,COSTA_CBLOCK=0 \
  -- --workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
timeout -k 10 300 python3 tools/ab_bench.py $O/c5N 2 c4:COSTA_LIB=$V/cbC4/lib/libcosta_amd.so \
  c2:COSTA_LIB=$V/cbC2/lib/libcosta_amd.so t128c4:COSTA_LIB=$V/cbT128C4/lib/libcosta_amd.so \
  wave:COSTA_TUNING=1,COSTA_CBLOCK=0 \
  -- --workload cfg5 --cfg5-op N --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra || exit 1
