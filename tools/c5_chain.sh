#!/bin/bash
# cfg5: destination order (sort 5) against destination order with source neighbours chained
# (sort 6): time and HBM traffic per launch, 'N' and 'T'
set -o pipefail
O=gpurun_out/${1:-c5chain}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
for s in 5 6; do
  for op in N T; do
    COSTA_TINY_SORT=$s timeout -k 10 200 $B --cfg5-op $op > $O/s$s.$op.json 2> $O/s$s.$op.err || exit 1
    for c in FETCH_SIZE WRITE_SIZE; do
      COSTA_TINY_SORT=$s timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_s${s}_${op}_$c -o p --output-format csv -- $B --steps 3 --cfg5-op $op > $O/pmc_s${s}_${op}_$c.log 2>&1 || exit 1
    done
  done
done
