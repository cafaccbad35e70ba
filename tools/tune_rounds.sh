#!/bin/bash
# Exchange rounds on one GPU: BASELINE cfg 2 through PACK -> RCCL self send/recv -> UNPACK
# (COSTA_LOOPBACK=1 routes every tile through the exchange) with COSTA_EXCHANGE_ROUNDS 1 / 4 / 8,
# interleaved twice.  Output: gpurun_out/<tag>/rounds.log
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-rounds}
mkdir -p "$OUT"
for rep in 1 2; do
    for R in 1 4 8; do
        COSTA_LOOPBACK=1 COSTA_EXCHANGE_ROUNDS=$R timeout -k 10 300 python3 bench.py --steps 20 \
            --warmup 3 --no-cpu-baseline --no-e2e > "$OUT/run.log" 2>&1 \
            || { echo "run failed: R=$R"; tail -5 "$OUT/run.log"; exit 3; }
        python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], 'value', d['value'], 'ms/step', d['ms_per_step'], 'phases', d['phase_ms_per_step'])" \
            "$OUT/run.log" "rep$rep rounds=$R" | tee -a "$OUT/rounds.log"
    done
done
