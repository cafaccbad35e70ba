#!/bin/bash
# r5 session r: the headline's placement mode against how the destination is allocated
# (torch / hipMalloc / physically contiguous), tools/alloc_probe.py
set -o pipefail
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 300 python3 -u tools/alloc_probe.py 4 > $O/alloc.txt 2>&1 || exit 1
