#!/bin/bash
# r6 final check, part b: cfg 5 'N' / 'T' and cfg 3 / cfg 4 kernel traces and HBM traffic passes
# (tools/c5_pmc.sh, tools/c34_prof.sh) -> profiles/r6z; read bytes by request size of cfg 2 and
# cfg 5 (tools/pmc_bytes.py)
set -o pipefail
tools/c5_pmc.sh r6z_c5pmc || exit 1
tools/c34_prof.sh r6z_c34 || exit 1
O=gpurun_out/r6z_bytes
mkdir -p $O
export TMPDIR=/tmp
P="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum"
B="--steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra"
for w in "cfg2:" "N:--workload cfg5 --cfg5-op N" "T:--workload cfg5 --cfg5-op T"; do
  n=${w%%:*}; a=${w#*:}
  timeout -s KILL 200 rocprofv3 --pmc $P -d $O/bytes_$n -o p --output-format csv -- python3 bench.py $a $B > $O/bytes_$n.log 2>&1 || exit 1
  echo "== $n" >> $O/bytes_summary.txt
  python3 tools/pmc_bytes.py $O/bytes_$n $([ $n = T ] && echo 2147483648 || ([ $n = N ] && echo 1073741824 || echo 2147483648)) >> $O/bytes_summary.txt 2>&1
done
