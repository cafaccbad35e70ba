#!/bin/bash
# r5 session g: the headline's two rates by physical placement (tools/pairs_probe.py: 8 pairs of
# separately allocated buffers in one process), and counter passes over the same probe whose
# dispatches split by duration into the fast and the slow placement (tools/pmc_modes.py)
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/pairs_probe.py 8 2 > $O/pairs.txt 2>&1 || exit 1
i=0
for set in "TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum GRBM_GUI_ACTIVE" \
           "TCC_EA0_RDREQ_GMI_CREDIT_STALL_sum TCC_EA0_WRREQ_GMI_CREDIT_STALL_sum TCC_EA0_RDREQ_IO_CREDIT_STALL_sum TCC_EA0_WRREQ_IO_CREDIT_STALL_sum GRBM_GUI_ACTIVE" \
           "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_WRITE_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE" \
           "TCC_TAG_STALL_sum TCC_EA0_WRREQ_STALL_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_PENDING_STALL_CYCLES_sum GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 200 rocprofv3 --pmc $set -d $O/p$i -o p$i --output-format csv -- python3 tools/pairs_probe.py 8 1 > $O/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/p$i.log; exit 1; }
done
