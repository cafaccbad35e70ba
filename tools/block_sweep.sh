#!/bin/bash
# 16384^2 'T' (alpha=1, beta=0) kernel rate over element types and block sizes, default library
set -u
cd "${GRAFT_REPO_ROOT:-.}"
out=gpurun_out/blocks/blocks.log
mkdir -p gpurun_out/blocks
: > $out
for cfg in "f64 16384 32 0" "f64 16384 64 0" "f64 16384 96 0" "f64 16384 128 0" "f64 16384 256 0" \
           "f32 16384 32 0" "f32 16384 64 0" "f32 16384 128 0" "f32 16384 256 0" \
           "c128 16384 32 0" "c128 16384 64 0" "c128 16384 128 0" "c64 16384 64 0" "c64 16384 128 0"; do
  timeout -k 10 120 python3 tools/order_probe.py $cfg 10 >> $out 2>/dev/null || { echo "fail $cfg" >> $out; exit 1; }
done
