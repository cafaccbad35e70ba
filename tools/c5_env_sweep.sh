#!/bin/bash
# cfg 5 probe (tools/c5_order_probe.py) under environment settings, one process each, 2 reps:
#   tools/c5_env_sweep.sh TAG "COSTA_TINY_SORT=1" "COSTA_TINY_SORT=2 COSTA_TINY_K=2" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=gpurun_out/$1/c5_env.log
shift
mkdir -p "$(dirname "$L")"
: > "$L"
for rep in 1 2; do
    for spec in "$@"; do
        for op in N T; do
            env $spec timeout -k 10 120 python3 tools/c5_order_probe.py $op 2>/dev/null \
                | sed "s/^{/{\"env\": \"$spec\", /" | grep '^{' >> "$L" || exit 1
        done
    done
done
cat "$L"
