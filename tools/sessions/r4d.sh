#!/bin/bash
# r4 session d: transposes by element size and matrix size (where c128 loses), and the PCIe
# behaviour the direct-download host pipeline would rely on
set -o pipefail
O=gpurun_out/r4d
mkdir -p $O
for a in "c128 8192 128 1.0" "c128 16384 128 1.0" "c128 16384 128 0.0" "f64 16384 128 1.0" "f64 32768 128 1.0" "c64 16384 128 1.0" "c64 32768 128 1.0" "f64 23168 128 1.0" "c128 16384 256 1.0" "c128 16384 64 1.0"; do
  timeout -k 10 200 python3 tools/order_probe.py $a 10 >> $O/sizes.txt 2>> $O/sizes.err || exit 1
done
timeout -k 10 200 tools/pcie_probe 2048 > $O/pcie.log 2>&1 || exit 1
