#!/bin/bash
# r5 session ao: the headline's bare access pattern with other store cache policies (libcosta_ceiling
# kinds 200-205: nt, default, sc1, sc1 nt, sc0 nt, sc0 sc1 nt), per buffer pair
set -o pipefail
O=gpurun_out/r5ao
mkdir -p $O
timeout -k 10 500 python3 -u tools/pattern_probe.py 6 pol > $O/policies.txt 2>&1 || exit 1
