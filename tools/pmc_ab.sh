#!/bin/bash
# Counter passes (one rocprofv3 --pmc run each, within the per-block limits of MI355X_MICROARCH.md)
# of one bench workload under several environment settings, for an A/B of where the time goes:
# texture-address / data units, L1 (TCP) requests and stalls, instruction counts.
#   tools/pmc_ab.sh OUTDIR 'label:ENV=V ENV=V' ... -- <bench args>
# summary: python3 tools/pmc_summary.py OUTDIR/<label> per setting
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1
shift
SETS=()
while [ "$1" != "--" ]; do SETS+=("$1"); shift; done
shift
mkdir -p "$OUT"
export TMPDIR=/tmp
PASSES=("TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
        "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_ADDR_STALLED_BY_TD_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE"
        "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE")
for s in "${SETS[@]}"; do
    label=${s%%:*}
    envs=${s#*:}
    i=0
    for set in "${PASSES[@]}"; do
        i=$((i + 1))
        mkdir -p "$OUT/$label"
        env $envs timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/$label/p$i" -o p$i --output-format csv -- python3 bench.py "$@" \
            > "$OUT/$label/p$i.log" 2>&1
        rc=$?
        echo "$label pass $i rc=$rc: $set"
        [ $rc -ne 0 ] && { tail -3 "$OUT/$label/p$i.log"; exit $rc; }
    done
done
exit 0
