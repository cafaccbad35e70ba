#!/bin/bash
# A/B of library builds and env knobs on one GPU lease (tuning, not product):
#   tools/ab_bench.sh OUTDIR "label|ENV=.. ENV2=..|bench args" ...
# Each entry runs `python3 bench.py --no-cpu-baseline --no-e2e <bench args>` with the env
# settings (COSTA_LIB=build/variants/<name>/libcosta_amd.so selects a tuning build) under its own
# time limit and prints value, kernel ms and roofline fraction.  Stops at the first crash.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=$1
shift
mkdir -p "$OUT"
for spec in "$@"; do
    IFS='|' read -r label envs args <<< "$spec"
    log="$OUT/$label.log"
    env $envs timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-e2e $args > "$log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then
        echo "$label rc=$rc"; tail -3 "$log"
        [ $rc -ne 1 ] && exit $rc
        continue
    fi
    python3 - "$label" "$log" <<'PY'
import json, sys
label, log = sys.argv[1], sys.argv[2]
d = [json.loads(l) for l in open(log) if l.startswith("{")][-1]
r = d["roofline"]
print(f"{label:28s} value {d['value']:8.1f} GB/s  step {d['ms_per_step']:.4f} ms  kernel {r['avg_launch_ms']:.4f} ms "
      f"{r['achieved']:8.1f} GB/s frac {r['frac']:.4f}")
PY
done
