#!/bin/bash
# r5 session ad: the shipped 4-group XCD chunks for transposing destination-block lists --
# cblock / cfg 5 / tile tests, cfg 5 'N' / 'T' bench lines, kernel traces and HBM traffic passes
# (tools/c5_pmc.sh) -> profiles/r5f2 (cfg 5 files)
set -o pipefail
O=gpurun_out/r5f2
mkdir -p $O
PT="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_cblock.py tests/test_gpu_cfg5.py tests/test_gpu_tiles.py > $O/pytest_c5.txt 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op N --steps 10 --no-cpu-baseline > $O/c5N.json 2> $O/c5N.err || exit 1
timeout -k 10 300 python3 bench.py --workload cfg5 --cfg5-op T --steps 10 --no-cpu-baseline > $O/c5T.json 2> $O/c5T.err || exit 1
tools/c5_pmc.sh r5f2_c5pmc || exit 1
