#!/bin/bash
# cfg 5 'N' / 'T' HBM traffic (FETCH_SIZE, WRITE_SIZE passes, one rocprofv3 run each) and a
# kernel trace of each; summaries by tools/pmc_brief.py (alg bytes: 'N' 2^31, 'T' 3 * 2^30)
set -o pipefail
O=gpurun_out/${1:-c5pmc}
mkdir -p $O
export TMPDIR=/tmp
for op in N T; do
  alg=$([ $op = N ] && echo 2147483648 || echo 3221225472)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$op -o trace --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op $op --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-extra > $O/prof_$op.log 2>&1 || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_${op}_$c -o p --output-format csv -- python3 bench.py --workload cfg5 --cfg5-op $op --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/pmc_${op}_$c.log 2>&1 || exit 1
    python3 tools/pmc_brief.py $O/pmc_${op}_$c $alg >> $O/summary_$op.txt 2>&1
  done
done
