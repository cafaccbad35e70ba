#!/bin/bash
# SQ / SPI / TA counter passes (one rocprofv3 --pmc run each, within the per-block slot limits of
# MI355X_MICROARCH.md) over one bench workload: occupancy (SQ_LEVEL_WAVES / SQ_BUSY_CYCLES),
# where wave time goes (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY), and whether the
# dispatcher or the texture-address path holds waves back.
#   tools/pmc_sq.sh OUTDIR -- <bench args>
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1
shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES GRBM_GUI_ACTIVE" \
           "SPI_RA_REQ_NO_ALLOC_CSN SPI_RA_WAVE_SIMD_FULL_CSN TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o p$i --output-format csv -- python3 bench.py "$@" \
        > "$OUT/p$i.log" 2>&1
    rc=$?
    echo "pass $i rc=$rc: $set"
    [ $rc -ne 0 ] && { tail -3 "$OUT/p$i.log"; exit $rc; }
done
exit 0
