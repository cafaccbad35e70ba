#!/bin/bash
# r5 session am: transposing access patterns of other fp64 sub-tile geometries without LDS
# (tools/pattern_probe.py, libcosta_ceiling kinds 100+): both sides / flat loads / flat stores
set -o pipefail
O=gpurun_out/r5am
mkdir -p $O
timeout -k 10 500 python3 -u tools/pattern_probe.py 6 > $O/patterns.txt 2>&1 || exit 1
