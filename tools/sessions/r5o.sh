#!/bin/bash
# r5 session o: counters of cfg 5 'T' on the destination-block groups (cblock_kernel): occupancy and
# wait shares, instruction mix and LDS conflicts, texture-path load, HBM traffic
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --workload cfg5 --cfg5-op T --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-extra"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/trace -o trace --output-format csv -- $B > $O/trace.log 2>&1 || exit 1
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LEVEL_WAVES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
           "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i + 1))
  timeout -s KILL 150 rocprofv3 --pmc $set -d $O/p$i -o p$i --output-format csv -- $B > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
