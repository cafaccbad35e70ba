#!/bin/bash
# r4 session zm: the default bench line with the extended copy ceiling
set -o pipefail
O=gpurun_out/r4zm
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
