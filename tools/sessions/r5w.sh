#!/bin/bash
# r5 session w: copy shapes with fewer loads a thread in flight.  cfg 3's copy slice on fp64
# tuning builds (COSTA_F64_COPY 2: 512 threads x 2 loads on 128 x 16 sub-tiles, 4: 512 x 1 on
# 128 x 8, 5: 256 x 2 on 128 x 8, 6: 1024 x 2 on 128 x 32) against the shipped 256 x 32 loads;
# then side by side (tools/libs_probe.py, op N) fp64 beta = 0 / 1.5, fp32, c64, c128 with every
# copy shape at 2 loads a thread (cps)
set -o pipefail
O=gpurun_out/r5w
mkdir -p $O
V=gpuvar
timeout -k 10 900 python3 tools/ab_bench.py $O/c3 2 shipped: cp2:COSTA_LIB=$V/cp2/lib/libcosta_amd.so \
  cp4:COSTA_LIB=$V/cp4/lib/libcosta_amd.so cp5:COSTA_LIB=$V/cp5/lib/libcosta_amd.so \
  cp6:COSTA_LIB=$V/cp6/lib/libcosta_amd.so \
  -- --workload cfg3 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extra || exit 1
L="shipped=costa_amd/lib/libcosta_amd.so cps=$V/cps/lib/libcosta_amd.so"
PROBE_OP=N PROBE_DT=f64 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/f64_N.txt 2>&1 || exit 1
PROBE_OP=N PROBE_DT=f64 PROBE_BETA=1.5 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/f64_N_beta.txt 2>&1 || exit 1
PROBE_OP=N PROBE_DT=f32 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/f32_N.txt 2>&1 || exit 1
PROBE_OP=N PROBE_DT=c64 PROBE_B=128 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/c64_N.txt 2>&1 || exit 1
PROBE_OP=N PROBE_DT=c128 PROBE_B=128 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/c128_N.txt 2>&1 || exit 1
