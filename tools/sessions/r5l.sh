#!/bin/bash
# r5 session l: store orders side by side on the same buffers (tools/libs_probe.py): fp64 headline
# (shipped / st8 / st9 / st10), fp32 16384^2 256^2 blocks 'T', c128 16384^2 128^2 'T' alpha, beta
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
V=gpuvar
L="shipped=costa_amd/lib/libcosta_amd.so st9=$V/st9/lib/libcosta_amd.so st10=$V/st10/lib/libcosta_amd.so"
timeout -k 10 300 python3 tools/libs_probe.py 8 $L st8=$V/st8/lib/libcosta_amd.so > $O/f64.txt 2>&1 || exit 1
PROBE_DT=f32 timeout -k 10 200 python3 tools/libs_probe.py 6 $L > $O/f32.txt 2>&1 || exit 1
PROBE_DT=c128 PROBE_B=128 PROBE_BETA=1.25 timeout -k 10 300 python3 tools/libs_probe.py 4 $L > $O/c128.txt 2>&1 || exit 1
