#!/bin/bash
# r5 session k: store orders side by side on the same buffers (tools/libs_probe.py): shipped, st7
# (a column pair's two chunks stored at once by two wavefronts), st8 (the same with LDS-DMA
# staging), st9 (a wavefront's own column pairs, chunks back to back), st1 (LDS-DMA)
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
V=gpuvar
timeout -k 10 300 python3 tools/libs_probe.py 8 shipped=costa_amd/lib/libcosta_amd.so st7=$V/st7/lib/libcosta_amd.so \
  st8=$V/st8/lib/libcosta_amd.so st9=$V/st9/lib/libcosta_amd.so st1=$V/st1/lib/libcosta_amd.so \
  > $O/libs.txt 2>&1 || exit 1
