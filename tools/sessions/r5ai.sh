#!/bin/bash
# r5 session ai: the fp64 transposing shape at 1024 threads (4 loads a thread) held to 64 VGPRs so
# that two workgroups fit a CU (tuning build gpuvar/h1024, COSTA_F64_TR1024) side by side with
# the shipped 512 threads: the headline (6 pairs), 128^2 blocks, beta != 0
set -o pipefail
O=gpurun_out/r5ai
mkdir -p $O
L="shipped=costa_amd/lib/libcosta_amd.so h1024=gpuvar/h1024/lib/libcosta_amd.so"
timeout -k 10 400 python3 -u tools/libs_probe.py 6 $L > $O/f64_T.txt 2>&1 || exit 1
PROBE_B=128 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/f64_T_b128.txt 2>&1 || exit 1
PROBE_BETA=1.5 timeout -k 10 300 python3 -u tools/libs_probe.py 3 $L > $O/f64_T_beta.txt 2>&1 || exit 1
