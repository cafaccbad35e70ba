#!/bin/bash
# GPU box (tuning, not product): copy lists on the large shape (tools/copy_probe.py, every element
# type, beta = 0 and beta != 0) and BASELINE cfg 3's copy slice, default library against the
# copy-shape variants under build/variants/ (tools/tiny_variants.sh)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-copy_shape_ab}
mkdir -p "$OUT"
timeout -k 10 300 python3 tools/copy_probe.py 10 > "$OUT/probe_default.log" 2>&1 || exit $?
for d in build/variants/*/; do
  n=$(basename "$d")
  COSTA_LIB=${d}libcosta_amd.so timeout -k 10 300 python3 tools/copy_probe.py 10 > "$OUT/probe_$n.log" 2>&1 || exit $?
done
for f in "$OUT"/probe_*.log; do echo "-- $f"; grep copy "$f" | sed 's/GB.*//'; done
specs=("c3_default||--workload cfg3 --steps 10 --warmup 2")
for d in build/variants/*/; do
  n=$(basename "$d")
  specs+=("c3_${n}|COSTA_LIB=${d}libcosta_amd.so|--workload cfg3 --steps 10 --warmup 2")
done
specs+=("c3_default_b||--workload cfg3 --steps 10 --warmup 2")
bash tools/ab_bench.sh "$OUT/ab" "${specs[@]}"
