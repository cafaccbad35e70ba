#!/bin/bash
# r5 session s: costa_amd.contiguous_pool() checked step by step (tools/pool_check.py), then
# torch-allocated (A, C) pairs against pairs from the pool (physically contiguous segments), the
# headline transpose on each (tools/alloc_probe.py pairs)
set -o pipefail
O=gpurun_out/r5s
mkdir -p $O
timeout -k 10 120 python3 -X faulthandler -u tools/pool_check.py > $O/pool_check.txt 2>&1 || exit 1
timeout -k 10 300 python3 -X faulthandler -u tools/alloc_probe.py pairs 5 > $O/pairs.txt 2>&1 || exit 1
