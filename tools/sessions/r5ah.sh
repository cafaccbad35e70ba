#!/bin/bash
# r5 session ah: the transposes' store phase at raised wave priority (s_setprio 1 / 3 after the
# barrier of full sub-tiles; tuning builds gpuvar/pr1, pr3, tile_kernels.hip COSTA_TR_PRIO) side by
# side with the shipped kernel: the fp64 headline (6 pairs) and cfg 4's c128 16384^2
set -o pipefail
O=gpurun_out/r5ah
mkdir -p $O
V=gpuvar
L="shipped=costa_amd/lib/libcosta_amd.so pr1=$V/pr1/lib/libcosta_amd.so pr3=$V/pr3/lib/libcosta_amd.so"
timeout -k 10 400 python3 -u tools/libs_probe.py 6 $L > $O/f64_T.txt 2>&1 || exit 1
PROBE_DT=c128 PROBE_B=128 PROBE_BETA=1.25 timeout -k 10 400 python3 -u tools/libs_probe.py 3 $L > $O/c128_T.txt 2>&1 || exit 1
PROBE_DT=f32 timeout -k 10 400 python3 -u tools/libs_probe.py 3 $L > $O/f32_T.txt 2>&1 || exit 1
