#!/bin/bash
# One GPU-box session: smoke -> GPU parity tests -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; the script stops at the first crash/timeout
# (test failures, exit 1, are reported but do not stop it).
#   usage: tools/gpu_check.sh [tag]      outputs under gpurun_out/<tag>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    echo "== $name: $*"
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    tail -5 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
        echo "stopping after $name (rc=$rc)"
        exit $rc
    fi
}

rocm-smi --showproductname > "$OUT/gpu.txt" 2>&1 || true
nproc > "$OUT/nproc.txt"; lscpu | grep -E "Model name|^CPU\(s\)" >> "$OUT/nproc.txt"
step smoke 400 python3 -c "import __graft_entry__ as g; g.smoke()"
step pytest_gpu 900 python3 -u -m pytest tests -m gpu -q --maxfail=20 --timeout 120 --timeout-method thread
step bench 600 python3 bench.py --steps 20 --warmup 3
step rocprof_trace 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o trace --output-format csv \
    -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-e2e
if [ "${PMC:-1}" = "1" ]; then
    step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/pmc_fetch" -o fetch --output-format csv \
        -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e
    step pmc_write 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/pmc_write" -o write --output-format csv \
        -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e
fi
if [ "${CFG5:-1}" = "1" ]; then
    for op in N T; do
        C5="python3 bench.py --workload cfg5 --cfg5-op $op --no-cpu-baseline --no-e2e"
        step c5${op}_bench 300 $C5 --steps 20 --warmup 3
        step c5${op}_rocprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/c5${op}_prof" -o trace \
            --output-format csv -- $C5 --steps 10 --warmup 2
        if [ "${PMC:-1}" = "1" ]; then
            step c5${op}_pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$OUT/c5${op}_pmc_fetch" -o fetch \
                --output-format csv -- $C5 --steps 5 --warmup 1
            step c5${op}_pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$OUT/c5${op}_pmc_write" -o write \
                --output-format csv -- $C5 --steps 5 --warmup 1
        fi
    done
fi
echo "done"
