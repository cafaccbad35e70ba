#!/bin/bash
# r5 session aq: write-side counters of the headline transpose, its bare pattern (kind 5), its
# transposed stores alone (kind 8) and the one-vector strided copy (kind 4), one process
# (tools/pairs_probe.py, 2 pairs, 1 round), one rocprofv3 --pmc pass of 4 TCC counters + GRBM
set -o pipefail
O=gpurun_out/r5aq
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_LEVEL_sum GRBM_GUI_ACTIVE -d $O/pw -o p --output-format csv -- python3 tools/pairs_probe.py 2 1 > $O/pw.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE -d $O/pr -o p --output-format csv -- python3 tools/pairs_probe.py 2 1 > $O/pr.log 2>&1 || exit 1
