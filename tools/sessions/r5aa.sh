#!/bin/bash
# r5 session aa: 1024-thread variants of other transposing shapes side by side (tools/libs_probe.py,
# op T, 16384^2, tuning build gpuvar/thr): fp32 128 x 128 large shape (256^2 blocks), fp64 and c64
# square 64 x 64 shapes (64^2 blocks)
set -o pipefail
O=gpurun_out/r5aa
mkdir -p $O
L="shipped=costa_amd/lib/libcosta_amd.so thr=gpuvar/thr/lib/libcosta_amd.so"
PROBE_DT=f32 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/f32_T.txt 2>&1 || exit 1
PROBE_DT=f64 PROBE_B=64 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/f64_T_b64.txt 2>&1 || exit 1
PROBE_DT=c64 PROBE_B=64 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/c64_T_b64.txt 2>&1 || exit 1
