#!/bin/bash
# Tuning builds (not product) of libcosta_amd.so with other wavefront-path constants:
#   tools/tiny_variants.sh NAME "-DCOSTA_TINY_BYTES=32 -DCOSTA_TINY_WAVES_TR=4" ...
# -> build/variants/NAME/libcosta_amd.so, loaded with COSTA_LIB=<that path>.
set -eu
cd "$(dirname "$0")/../costa_amd/csrc"
make -j8 > /dev/null
OBJ="../lib/obj/layout.o ../lib/obj/plan.o ../lib/obj/engine.o ../lib/obj/capi.o ../lib/obj/host_pipe.o ../lib/obj/relabel.o ../lib/obj/device_plan.o"
while [ $# -ge 2 ]; do
    name=$1 defs=$2
    shift 2
    out=../../build/variants/$name
    mkdir -p "$out"
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -ffp-contract=off -I../../include -I/opt/rocm/include \
        -x hip --offload-arch=gfx950 -munsafe-fp-atomics $defs -c tile_kernels.hip -o "$out/tile_kernels.o" &
done
wait
for d in ../../build/variants/*/; do
    /opt/rocm/bin/hipcc -shared -fPIC -pthread --offload-arch=gfx950 -o "$d/libcosta_amd.so" $OBJ \
        "$d/tile_kernels.o" -L/opt/rocm/lib -lamdhip64 -lrccl -Wl,-soname,libcosta_amd.so
done
ls ../../build/variants/
