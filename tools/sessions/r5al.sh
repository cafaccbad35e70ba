#!/bin/bash
# r5 session al: is the headline's placement bimodality in its access pattern alone?  Per buffer
# pair: the transpose, the one-vector strided copy and the transpose's loads / stores without
# LDS (libcosta_ceiling kind 5), 8 pairs, 2 rounds (tools/pairs_probe.py)
set -o pipefail
O=gpurun_out/r5al
mkdir -p $O
timeout -k 10 400 python3 -u tools/pairs_probe.py 8 2 > $O/pairs.txt 2>&1 || exit 1
