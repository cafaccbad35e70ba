#!/bin/bash
# r5 session ap: the headline's bare access pattern with other sub-tile orders (libcosta_ceiling
# kinds 300-305), per buffer pair
set -o pipefail
O=gpurun_out/r5ap
mkdir -p $O
timeout -k 10 500 python3 -u tools/pattern_probe.py 6 ord > $O/orders.txt 2>&1 || exit 1
