#!/bin/bash
# r4 session zg: the pageable end-to-end pipeline with cached or streaming host stores, slot sizes
set -o pipefail
O=gpurun_out/r4zg
mkdir -p $O
timeout -k 10 900 python3 -u tools/host_pipe_probe.py nt > $O/nt.txt 2> $O/err.txt || exit 1
