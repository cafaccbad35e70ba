#!/bin/bash
# cfg 2: destination order (3) against f-neighbour pairs / quads (4 / 5), alternating, one lease
set -o pipefail
O=gpurun_out/${1:-c2order}
mkdir -p $O
for k in 1 2 3; do
  for m in 3 4 5; do
    COSTA_LARGE_SORT=$m timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-extra > $O/s$m.$k.json 2> $O/s$m.$k.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_launch_ms'], d['verified'])" $O/s$m.$k.json "sort=$m" | tee -a $O/summary.txt
  done
done
