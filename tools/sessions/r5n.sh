#!/bin/bash
# r5 session n: destination band walks side by side (tools/libs_probe.py, tuning builds of
# engine.hpp kDstOrderVariant: 1 boustrophedon, 2 band pairs, 3 skewed starts, 4 band quads) on
# the fp64 headline; cfg 4's 32768^2 c128 slice with LDS-DMA + column-pair stores (st10)
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
V=gpuvar
timeout -k 10 300 python3 tools/libs_probe.py 6 shipped=costa_amd/lib/libcosta_amd.so ord1=$V/ord1/lib/libcosta_amd.so \
  ord2=$V/ord2/lib/libcosta_amd.so ord3=$V/ord3/lib/libcosta_amd.so ord4=$V/ord4/lib/libcosta_amd.so > $O/f64_orders.txt 2>&1 || exit 1
PROBE_DT=c128 PROBE_N=32768 PROBE_B=128 PROBE_BETA=1.25 timeout -k 10 300 python3 tools/libs_probe.py 2 \
  shipped=costa_amd/lib/libcosta_amd.so st10=$V/st10/lib/libcosta_amd.so > $O/c128_32768.txt 2>&1 || exit 1
