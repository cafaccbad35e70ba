#!/bin/bash
# Wave-path knobs on cfg5 ('N', 'T') and cfg2: COSTA_WAVE_POLICY x COSTA_TINY_SORT x assignment.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-wave}
mkdir -p "$OUT"
run() {  # run <workload> <op> <policy> <sort> <chunked> <k>
  local tag="$1.$2.p$3.s$4.c$5.k$6"
  COSTA_WAVE_POLICY=$3 COSTA_TINY_SORT=$4 COSTA_TINY_CHUNKED=$5 COSTA_TINY_K=$6 timeout -k 10 300 \
      python3 bench.py --workload $1 --cfg5-op $2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e \
      > "$OUT/$tag.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "stop: $tag rc=$rc"; tail -5 "$OUT/$tag.log"; exit $rc; fi
  python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); print(sys.argv[2], d['value'], d['kernel_node_GBps'])" "$OUT/$tag.log" "$tag"
}
for op in N T; do
  run cfg5 $op 1 2 0 1
  run cfg5 $op 2 2 0 1
  run cfg5 $op 0 2 0 1
  run cfg5 $op 1 2 1 4
  run cfg5 $op 1 1 0 1
  run cfg5 $op 1 0 0 1
done
run pxtran T 1 2 0 1
run pxtran T 2 2 0 1
