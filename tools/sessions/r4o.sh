#!/bin/bash
# r4 session o: is the headline's in-run kernel time different with the CPU baseline leg first?
set -o pipefail
O=gpurun_out/r4o
mkdir -p $O
for r in 1 2 3; do
  for v in full nocpu; do
    a=""; [ $v = nocpu ] && a="--no-cpu-baseline"
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-e2e --no-extra $a > $O/$v$r.json 2> $O/$v$r.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['roofline']['copy_ceiling']['strided_nt_1KiB_segments']['ms'])" $O/$v$r.json $v >> $O/summary.txt
  done
done
