#!/bin/bash
# r5 session t: far-apart destination band walks side by side on the fp64 headline (tuning builds
# of engine.hpp kDstOrderVariant: 5 halves interleaved per sub-tile, 6 quarters, 7 reversed,
# 8 halves band by band), 8 pairs, odd pairs physically contiguous (both placement modes)
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
V=gpuvar
PROBE_ALLOC=mix timeout -k 10 300 python3 -u tools/libs_probe.py 8 shipped=costa_amd/lib/libcosta_amd.so \
  ord5=$V/ord5/lib/libcosta_amd.so ord6=$V/ord6/lib/libcosta_amd.so ord7=$V/ord7/lib/libcosta_amd.so \
  ord8=$V/ord8/lib/libcosta_amd.so > $O/f64_orders.txt 2>&1 || exit 1
