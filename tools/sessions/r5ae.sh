#!/bin/bash
# r5 session ae: the large-shape sub-tiles in chunks of k consecutive work items per XCD (tuning
# builds gpuvar/tk{2,4,8}, tile_kernels.hip COSTA_TK_XK) side by side with the shipped
# round-robin dispatch: the fp64 headline (6 pairs) and cfg 4's c128 16384^2 (alpha, beta)
set -o pipefail
O=gpurun_out/r5ae
mkdir -p $O
V=gpuvar
L="shipped=costa_amd/lib/libcosta_amd.so tk2=$V/tk2/lib/libcosta_amd.so tk4=$V/tk4/lib/libcosta_amd.so tk8=$V/tk8/lib/libcosta_amd.so"
timeout -k 10 400 python3 -u tools/libs_probe.py 6 $L > $O/f64_T.txt 2>&1 || exit 1
PROBE_DT=c128 PROBE_B=128 PROBE_BETA=1.25 timeout -k 10 400 python3 -u tools/libs_probe.py 3 $L > $O/c128_T.txt 2>&1 || exit 1
PROBE_OP=N PROBE_B=128 timeout -k 10 400 python3 -u tools/libs_probe.py 3 $L > $O/f64_N.txt 2>&1 || exit 1
