#!/bin/bash
# r4 session zh: cfg 5's ceiling, the copy and the three-stream C = A + C of short runs
set -o pipefail
O=gpurun_out/r4zh
mkdir -p $O
timeout -k 10 200 tools/stride_probe runs > $O/runs.txt 2>&1 || exit 1
