#!/bin/bash
# cfg5 sweep: tiny-kernel waves per workgroup x bytes in flight per lane x XCD remap.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-wave2}
mkdir -p "$OUT"
run() {  # run <op> <waves> <bytes> <xcd>
  local tag="$1.w$2.b$3.x$4"
  COSTA_TINY_WAVES=$2 COSTA_TINY_BYTES=$3 COSTA_TINY_XCD=$4 timeout -k 10 300 \
      python3 bench.py --workload cfg5 --cfg5-op $1 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
      > "$OUT/$tag.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stop: $tag rc=$rc"; tail -5 "$OUT/$tag.log"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_node_GBps'])" "$OUT/$tag.log" "$tag"
}
for op in N T; do
  for x in 0 1; do
    for wb in "4 64" "2 64" "8 64" "4 32" "8 32" "4 128"; do run $op $wb $x; done
  done
done
