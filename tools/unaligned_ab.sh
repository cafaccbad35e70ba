#!/bin/bash
# GPU box: parity tests, then unaligned-column A/B on one lease (tuning, not product):
# the default library (policy 3: unaligned large ops on the large shape's element-wise path)
# against COSTA_WAVE_POLICY=2 (r2 classification, same kernels) and the r2 build
# (build/variants/novec with COSTA_WAVE_POLICY=2).
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
run pytest_gpu 900 python3 -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread
run unaligned_new 300 python3 tools/unaligned_probe.py 10
COSTA_WAVE_POLICY=2 run unaligned_pol2 300 python3 tools/unaligned_probe.py 10
COSTA_LIB=build/variants/novec/libcosta_amd.so COSTA_WAVE_POLICY=2 run unaligned_old 300 python3 tools/unaligned_probe.py 10
NV="COSTA_LIB=build/variants/novec/libcosta_amd.so COSTA_WAVE_POLICY=2"
bash tools/ab_bench.sh "$OUT/ab" \
    "c2_new||--steps 20 --warmup 3" \
    "c2_old|$NV|--steps 20 --warmup 3" \
    "c5N_new||--workload cfg5 --cfg5-op N --steps 20 --warmup 3" \
    "c5T_new||--workload cfg5 --cfg5-op T --steps 20 --warmup 3" \
    "c2_new_2||--steps 20 --warmup 3"
echo done
