#!/bin/bash
# r6 session m: cfg 5 'T' -- the XCD chunk size of transposing destination-block groups
# (COSTA_CB_CHUNK, default 4) and the column bands, time (alternating fresh processes) and read
# bytes by request size of each
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
export TMPDIR=/tmp
B="--workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra"
SETS=("c4:" "c8:COSTA_TUNING=1,COSTA_CB_CHUNK=8" "c16:COSTA_TUNING=1,COSTA_CB_CHUNK=16" "c32:COSTA_TUNING=1,COSTA_CB_CHUNK=32" "c64:COSTA_TUNING=1,COSTA_CB_CHUNK=64" "bands:COSTA_TUNING=1,COSTA_CB_BANDS=1")
timeout -k 10 900 python3 tools/ab_bench.py $O/ab 2 "${SETS[@]}" -- $B > $O/ab.log 2>&1 || exit 1
for s in "${SETS[@]}"; do
  label=${s%%:*}; envs=$(echo ${s#*:} | tr ',' ' ')
  env $envs timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum -d $O/b_$label -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op T --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/b_$label.log 2>&1 || exit 1
  echo "== $label" >> $O/bytes.txt
  python3 tools/pmc_bytes.py $O/b_$label 2147483648 >> $O/bytes.txt 2>&1
done
