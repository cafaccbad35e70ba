#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes for 4-byte wavefront accesses (tools/pmc_calib_tiny.py).
#   usage: tools/pmc_calib.sh [tag]      outputs under gpurun_out/<tag>/calib_*
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-calib}
mkdir -p "$OUT"
export TMPDIR=/tmp
for op in N T; do
    timeout -k 10 120 python3 tools/pmc_calib_tiny.py $op > "$OUT/calib_$op.log" 2>&1 || exit $?
    tail -1 "$OUT/calib_$op.log"
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 90 rocprofv3 --pmc $c -d "$OUT/calib_${op}_$c" -o c --output-format csv \
            -- python3 tools/pmc_calib_tiny.py $op > "$OUT/calib_${op}_$c.log" 2>&1 || exit $?
    done
done
echo done
