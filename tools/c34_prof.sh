#!/bin/bash
# BASELINE cfg 4 (pztranu c128 alpha, beta != 0, 128^2 blocks; 32768^2 single-GPU slice) and
# cfg 3 (pxgemr2d fp64 copy slice, 32768^2, 128^2 blocks): rocprofv3 kernel trace + stats and
# FETCH_SIZE / WRITE_SIZE passes (one rocprofv3 run per counter), summaries by pmc_brief.py.
#   tools/c34_prof.sh <tag> [extra bench args for cfg 4]
set -o pipefail
O=gpurun_out/${1:-c34}
shift
mkdir -p $O
export TMPDIR=/tmp
run() {  # name alg-bytes bench-args...
  local n=$1 alg=$2
  shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$n -o trace --output-format csv -- python3 bench.py "$@" --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-extra > $O/prof_$n.log 2>&1 || exit 1
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_${n}_$c -o p --output-format csv -- python3 bench.py "$@" --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-extra > $O/pmc_${n}_$c.log 2>&1 || exit 1
    python3 tools/pmc_brief.py $O/pmc_${n}_$c $alg >> $O/summary_$n.txt 2>&1
  done
}
# cfg 4 slice: 3 streams of 32768^2 c128 (A read, C read + written) = 51 539 607 552 B
run cfg4 51539607552 --workload cfg4 --edge 32768 "$@"
# cfg 3 copy slice: 2 streams of 32768^2 fp64 = 17 179 869 184 B
run cfg3 17179869184 --workload cfg3
