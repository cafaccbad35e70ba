#!/bin/bash
# r4 session zj: cfg 2's copy ceiling under other workgroup shapes (bytes in flight per workgroup)
set -o pipefail
O=gpurun_out/r4zj
mkdir -p $O
timeout -k 10 200 tools/stride_probe inflight > $O/inflight.txt 2>&1 || exit 1
timeout -k 10 200 python3 tools/order_probe.py f64 16384 256 0.0 20 >> $O/inflight.txt 2>> $O/err.txt || exit 1
