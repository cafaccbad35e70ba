#!/bin/bash
# cfg 5 wavefront budgets under the default XCD remap (tools/c5_order_probe.py, one process each)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=gpurun_out/${1:-r11}/c5_budget.log
mkdir -p "$(dirname "$L")"
: > "$L"
for rep in 1 2; do
    for cb in ${CB:-8192 4096 16384}; do
        COSTA_TINY_COPY_BUDGET=$cb timeout -k 10 120 python3 tools/c5_order_probe.py N 2>/dev/null \
            | sed "s/^{/{\"copy_budget\": $cb, /" | grep '^{' >> "$L" || exit 1
    done
    for lb in ${LB:-8192 6144 4096}; do
        COSTA_TINY_LDS_BUDGET=$lb timeout -k 10 120 python3 tools/c5_order_probe.py T 2>/dev/null \
            | sed "s/^{/{\"lds_budget\": $lb, /" | grep '^{' >> "$L" || exit 1
    done
done
cat "$L"
