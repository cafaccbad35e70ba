#!/bin/bash
# r5 session an: the default bench line after the ceiling library gained its probe kinds (the
# copy ceiling kinds 0-4 unchanged) -- a check that the line still carries every entry
set -o pipefail
O=gpurun_out/r5an
mkdir -p $O
timeout -k 10 480 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 1
