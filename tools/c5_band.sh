#!/bin/bash
# cfg5 'N': destination order (sort 5) against destination rows merged in bands of H (sort 7)
set -o pipefail
O=gpurun_out/${1:-c5band}
mkdir -p $O
export TMPDIR=/tmp
B="python3 bench.py --workload cfg5 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e"
run() {  # tag, env...
  local t=$1; shift
  env "$@" timeout -k 10 200 $B --cfg5-op N > $O/$t.json 2> $O/$t.err || return 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_launch_ms'], d['verified'])" $O/$t.json $t | tee -a $O/summary.txt
}
run s5 COSTA_TINY_SORT=5 && run h2 COSTA_TINY_SORT=7 COSTA_BAND_H=2 && run h3 COSTA_TINY_SORT=7 COSTA_BAND_H=3 &&
run h4 COSTA_TINY_SORT=7 COSTA_BAND_H=4 && run h8 COSTA_TINY_SORT=7 COSTA_BAND_H=8 && run s5b COSTA_TINY_SORT=5 || exit 1
for h in 2 4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    COSTA_TINY_SORT=7 COSTA_BAND_H=$h timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_h${h}_$c -o p --output-format csv -- $B --steps 3 --cfg5-op N > $O/pmc_h${h}_$c.log 2>&1 || exit 1
  done
done
