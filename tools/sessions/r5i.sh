#!/bin/bash
# r5 session i: the destination buffer's placement decides the headline's mode (r5h); the 8-pair
# distribution with default-policy stores (tuning build ntS0), destination panels of 64 / 32 KiB
# (COSTA_PANEL_ROWS), hint order (COSTA_LARGE_SORT=1), against the shipped kernel, 8 pairs each
set -o pipefail
O=gpurun_out/r5i
mkdir -p $O
P="timeout -k 10 150 python3 tools/pairs_probe.py 8 1"
$P > $O/pairs_shipped.txt 2>&1 || exit 1
COSTA_LIB=gpuvar/ntS0/lib/libcosta_amd.so $P > $O/pairs_ntS0.txt 2>&1 || exit 1
COSTA_TUNING=1 COSTA_PANEL_ROWS=8192 $P > $O/pairs_panel8192.txt 2>&1 || exit 1
COSTA_TUNING=1 COSTA_PANEL_ROWS=4096 $P > $O/pairs_panel4096.txt 2>&1 || exit 1
COSTA_TUNING=1 COSTA_LARGE_SORT=1 $P > $O/pairs_hint.txt 2>&1 || exit 1
