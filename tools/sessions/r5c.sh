#!/bin/bash
# r5 session c: what separates the headline transpose from the one-vector-per-thread copy of the
# same bytes (bench.py's copy ceiling, same process): L2 -> EA request queues and credit stalls,
# TA -> L2 latency, UTCL1 translation; one rocprofv3 --pmc pass per counter set (block limits of
# MI355X_MICROARCH.md), kernel trace + stats first
set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extra"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- $B > $O/trace.log 2>&1 || exit 1
i=0
for set in "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $set -d $O/p$i -o p$i --output-format csv -- $B > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
