#!/bin/bash
# cfg 2 kernel time in several fresh processes on one lease (placement spread), the counters
# the pool offers (for TLB / channel counters), and the unaligned-lld probe
set -o pipefail
O=gpurun_out/${1:-c2procs}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --list-avail > $O/list_avail.txt 2>&1 || true
for k in 1 2 3 4 5; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-extra > $O/bench$k.json 2> $O/bench$k.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('proc', sys.argv[2], d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])" $O/bench$k.json $k | tee -a $O/summary.txt
done
timeout -k 10 300 python3 tools/unaligned_probe.py 10 > $O/unaligned.log 2>&1
