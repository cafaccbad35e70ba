#!/bin/bash
# r4 session za: the three-stream ceiling of cfg 4 (reads A and C, writes C) against the copy
set -o pipefail
O=gpurun_out/r4za
mkdir -p $O
for i in 1 2 3; do timeout -k 10 120 tools/stride_probe three >> $O/three.txt 2>&1 || exit 1; done
timeout -k 10 200 python3 tools/order_probe.py c128 16384 128 1.0 10 >> $O/three.txt 2>> $O/err.txt || exit 1
timeout -k 10 200 python3 tools/order_probe.py c128 16384 128 0.0 10 >> $O/three.txt 2>> $O/err.txt || exit 1
