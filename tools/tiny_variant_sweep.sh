#!/bin/bash
# cfg 5 probe over the tuning builds of tools/tiny_variants.sh (one process per setting)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=gpurun_out/${1:-r11}/tiny_variants.log
mkdir -p "$(dirname "$L")"
: > "$L"
export COSTA_TINY_COPY_BYTES=${COSTA_TINY_COPY_BYTES:-64} COSTA_TINY_COPY_BUDGET=${COSTA_TINY_COPY_BUDGET:-4096}
for rep in 1 2; do
    for d in build/variants/*/; do
        v=$(basename "$d")
        COSTA_LIB=$PWD/$d/libcosta_amd.so timeout -k 10 120 python3 tools/c5_order_probe.py N 2>/dev/null \
            | sed "s/^{/{\"variant\": \"$v\", /" | grep '^{' >> "$L" || exit 1
        for lb in ${LB:-8192 4096}; do
            COSTA_TINY_LDS_BUDGET=$lb COSTA_LIB=$PWD/$d/libcosta_amd.so timeout -k 10 120 \
                python3 tools/c5_order_probe.py T 2>/dev/null \
                | sed "s/^{/{\"variant\": \"$v\", \"lds_budget\": $lb, /" | grep '^{' >> "$L" || exit 1
        done
    done
done
cat "$L"
