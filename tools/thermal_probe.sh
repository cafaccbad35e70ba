#!/bin/bash
# cfg 2 kernel time against the GPU's temperature history: back-to-back runs, a run after 60 s
# idle, runs right after a minute of cfg 5 'T' load; the temperatures rocm-smi reports between
set -o pipefail
O=gpurun_out/${1:-thermal}; mkdir -p $O
t() { rocm-smi --showtemp 2>/dev/null | grep -i "temp" | tr -s ' ' | head -6 | tr '\n' ';' >> $O/log.txt; echo >> $O/log.txt; }
b() { echo "== $1" >> $O/log.txt; t; timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-extra 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('kernel', d['roofline']['avg_launch_ms'], 'value', d['value'])" >> $O/log.txt || exit 1; }
b first
b second
b third
sleep 60
b after_60s_idle
for i in 1 2 3 4 5 6; do timeout -k 10 120 python3 bench.py --workload cfg5 --cfg5-op T --steps 400 --warmup 5 --no-cpu-baseline --no-e2e --no-extra > /dev/null 2>&1 || exit 1; done
b after_load
b after_load_2
