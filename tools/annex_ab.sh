#!/bin/bash
# cost of the Annex G recovery in the complex kernels: shipped library vs a naive-product build
set -o pipefail
O=gpurun_out/${1:-annexab}
mkdir -p $O
for k in 1 2; do
  for v in shipped noannex; do
    L=""; [ $v = noannex ] && L="COSTA_LIB=build/variants/noannex/libcosta_amd.so"
    env $L timeout -k 10 300 python3 bench.py --workload cfg4 --steps 10 --no-cpu-baseline > $O/c4_$v$k.json 2> $O/c4_$v$k.err || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['avg_launch_ms'], d['verified'])" $O/c4_$v$k.json $v | tee -a $O/summary.txt
  done
done
