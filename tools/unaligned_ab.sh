#!/bin/bash
# GPU box: parity tests, then the unaligned-column change A/B on one lease (tuning, not product):
# 16-byte vectors at dword alignment in the shapes + size-only classification (default build)
# against the r2 scheme (build/variants/novec: COSTA_UNALIGNED_VEC=0, COSTA_WAVE_POLICY=2).
#   usage: tools/unaligned_ab.sh TAG     (outputs under gpurun_out/TAG/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-ua}
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {  # run <name> <seconds> <cmd...>
    local name=$1 secs=$2
    shift 2
    timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc"; tail -4 "$OUT/$name.log"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name"; exit $rc; fi
}
run smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread
run unaligned_new 300 python3 tools/unaligned_probe.py 10
COSTA_LIB=build/variants/novec/libcosta_amd.so COSTA_WAVE_POLICY=2 run unaligned_old 300 python3 tools/unaligned_probe.py 10
NV="COSTA_LIB=build/variants/novec/libcosta_amd.so COSTA_WAVE_POLICY=2"
bash tools/ab_bench.sh "$OUT/ab" \
    "c2_new||--steps 20 --warmup 3" \
    "c5N_new||--workload cfg5 --cfg5-op N --steps 20 --warmup 3" \
    "c5N_old|$NV|--workload cfg5 --cfg5-op N --steps 20 --warmup 3" \
    "c5T_new||--workload cfg5 --cfg5-op T --steps 20 --warmup 3" \
    "c5T_old|$NV|--workload cfg5 --cfg5-op T --steps 20 --warmup 3" \
    "c5T_new_pol2|COSTA_WAVE_POLICY=2|--workload cfg5 --cfg5-op T --steps 20 --warmup 3" \
    "c5N_new_2||--workload cfg5 --cfg5-op N --steps 20 --warmup 3" \
    "c5T_new_2||--workload cfg5 --cfg5-op T --steps 20 --warmup 3" \
    "c2_old|$NV|--steps 20 --warmup 3"
echo done
