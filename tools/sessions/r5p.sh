#!/bin/bash
# r5 session p: cfg 4's 32768^2 c128 slice (alpha, beta) with other destination panel heights
# (engine.hpp kPanelBytes tuning builds: 96 / 192 / 256 KiB against the shipped 128), side by side
set -o pipefail
O=gpurun_out/r5p
mkdir -p $O
V=gpuvar
PROBE_DT=c128 PROBE_N=32768 PROBE_B=128 PROBE_BETA=1.25 timeout -k 10 400 python3 tools/libs_probe.py 2 \
  shipped=costa_amd/lib/libcosta_amd.so pan96=$V/pan96/lib/libcosta_amd.so pan192=$V/pan192/lib/libcosta_amd.so \
  pan256=$V/pan256/lib/libcosta_amd.so > $O/c128_32768.txt 2>&1 || exit 1
