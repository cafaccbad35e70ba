#!/bin/bash
# (The COSTA_SKEW / COSTA_LARGE_XCD / COSTA_UNALIGNED_ELEM knobs belonged to an r2c experiment
# that was measured slower and not kept in the library: DESIGN.md §3, profiles/r2c/unaligned/.)
# GPU box (tuning, not product): unaligned large ops under the shaped kernel's knobs
# (COSTA_SKEW, COSTA_LARGE_XCD, COSTA_UNALIGNED_ELEM; r2 build: build/variants/novec with
# COSTA_WAVE_POLICY=2), then cfg 2 / cfg 5 with the defaults.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ua}
mkdir -p "$OUT"
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 "$OUT/$name.log"; echo "stopping after $name"; exit $rc; fi
}
run pytest_tiles 300 python3 -u -m pytest tests/test_gpu_tiles.py -q -x --timeout 120 --timeout-method thread
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
run default 300 python3 tools/unaligned_probe.py 10
COSTA_SKEW=0 run noskew 300 python3 tools/unaligned_probe.py 10
COSTA_SKEW=0 COSTA_LARGE_XCD=0 run elem_only 300 python3 tools/unaligned_probe.py 10
COSTA_SKEW=1 COSTA_LARGE_XCD=0 run skew_noxcd 300 python3 tools/unaligned_probe.py 10
COSTA_SKEW=0 COSTA_LARGE_XCD=0 COSTA_UNALIGNED_ELEM=0 run strips 300 python3 tools/unaligned_probe.py 10
COSTA_LIB=build/variants/novec/libcosta_amd.so COSTA_WAVE_POLICY=2 run r2 300 python3 tools/unaligned_probe.py 10
bash tools/ab_bench.sh "$OUT/ab" "c2||--steps 20 --warmup 3" "c2_x2|COSTA_LARGE_XCD=2|--steps 20 --warmup 3" \
    "c5N||--workload cfg5 --cfg5-op N --steps 20 --warmup 3" "c5T||--workload cfg5 --cfg5-op T --steps 20 --warmup 3"
for f in default noskew elem_only skew_noxcd strips r2; do echo "-- $f"; grep lld "$OUT/$f.log" | grep -v "lld 16384" | sed 's/GB.*//'; done
