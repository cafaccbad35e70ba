#!/bin/bash
# HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of 16384^2 'T' with leading dimensions off the
# 16-byte grid: fp32 both sides lld 16385, fp32 destination lld 16386, fp64 both sides 16385,
# and aligned fp32 for comparison; summaries by tools/pmc_brief.py
set -o pipefail
O=gpurun_out/${1:-skewpmc}
mkdir -p $O
export TMPDIR=/tmp
cat > $O/one.py <<'PY'
import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
import torch, costa_amd as costa
import unaligned_probe as u
costa.lib(); comm = costa.Comm.self(0)
dt = costa.FLOAT if sys.argv[1] == "f" else costa.DOUBLE
u.run(dt, 16384, 256, int(sys.argv[2]), 3, comm, int(sys.argv[3]))
PY
for cfg in "f 16385 16385" "f 16384 16386" "d 16385 16385" "f 16384 16384"; do
  tag=$(echo $cfg | tr ' ' '_')
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 200 rocprofv3 --pmc $c -d $O/$tag/$c -o p --output-format csv -- python3 $O/one.py $cfg > $O/$tag.$c.log 2>&1 || exit 1
    python3 tools/pmc_brief.py $O/$tag/$c >> $O/summary.txt 2>&1
  done
  echo "== $cfg" >> $O/summary.txt
done
