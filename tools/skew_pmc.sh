#!/bin/bash
# skew shape: granule sizes probe + HBM traffic of fp64 lld 16384 -> 16385 (destination unaligned)
set -o pipefail
O=gpurun_out/${1:-skewpmc}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 ./tools/partial_line_probe 10 > $O/plp.log 2>&1 || exit 1
cat > $O/one.py <<'PY'
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
import torch, costa_amd as costa
import unaligned_probe as u
costa.lib(); comm = costa.Comm.self(0)
u.run(costa.DOUBLE, 16384, 256, int(sys.argv[1]), 3, comm, int(sys.argv[2]))
PY
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c -d $O/pmc_dst_$c -o p --output-format csv -- python3 $O/one.py 16384 16385 > $O/pmc_dst_$c.log 2>&1 || exit 1
done
