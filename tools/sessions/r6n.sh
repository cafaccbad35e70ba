#!/bin/bash
# r6 session n: cfg 5 'T' XCD chunk sizes 4-16 (3 alternating reps), rocprofv3 kernel traces and
# read bytes by request size of 8, 12 and 16, the standard FETCH_SIZE / WRITE_SIZE traffic of 8 and 16
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
export TMPDIR=/tmp
B="--workload cfg5 --cfg5-op T --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-extra"
timeout -k 10 900 python3 tools/ab_bench.py $O/ab 3 "c4:" "c6:COSTA_TUNING=1,COSTA_CB_CHUNK=6" "c8:COSTA_TUNING=1,COSTA_CB_CHUNK=8" "c12:COSTA_TUNING=1,COSTA_CB_CHUNK=12" "c16:COSTA_TUNING=1,COSTA_CB_CHUNK=16" -- $B > $O/ab.log 2>&1 || exit 1
for c in 4 8 12 16; do
  env COSTA_TUNING=1 COSTA_CB_CHUNK=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t_c$c -o trace --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op T --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-extra > $O/t_c$c.log 2>&1 || exit 1
done
for c in 8 12 16; do
  env COSTA_TUNING=1 COSTA_CB_CHUNK=$c timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum -d $O/b_c$c -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op T --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/b_c$c.log 2>&1 || exit 1
  echo "== c$c" >> $O/bytes.txt
  python3 tools/pmc_bytes.py $O/b_c$c 2147483648 >> $O/bytes.txt 2>&1
done
for c in 8 16; do
  for k in FETCH_SIZE WRITE_SIZE; do
    env COSTA_TUNING=1 COSTA_CB_CHUNK=$c timeout -s KILL 120 rocprofv3 --pmc $k -d $O/pmc_c${c}_$k -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op T --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/pmc_c${c}_$k.log 2>&1 || exit 1
    echo "== c$c $k" >> $O/traffic.txt
    python3 tools/pmc_brief.py $O/pmc_c${c}_$k 3221225472 >> $O/traffic.txt 2>&1
  done
done
