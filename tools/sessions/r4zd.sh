#!/bin/bash
# r4 session zd: cfg 4's three-stream ceiling on the 32768^2 slice geometry
set -o pipefail
O=gpurun_out/r4zd
mkdir -p $O
for i in 1 2; do timeout -k 10 120 tools/stride_probe three 32768 >> $O/three32768.txt 2>&1 || exit 1; done
timeout -k 10 200 python3 tools/order_probe.py c128 32768 128 1.0 6 >> $O/three32768.txt 2>> $O/err.txt || exit 1
