#!/bin/bash
# Build a tuning variant of the library from the current sources with sed edits applied to
# tile_kernels.hip and engine.hpp: build/variants/<name>/lib/libcosta_amd.so (load it with COSTA_LIB=...).
#   tools/build_variant.sh <name> '<sed expression>' ['<sed expression>' ...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
V=${VARIANT_DIR:-$ROOT/build/variants}  # VARIANT_DIR: a directory that travels to the GPU box
name=$1
shift
rm -rf "$V/$name"
mkdir -p "$V/$name"
ln -sfn "$ROOT/include" "$V/include"
cp -r "$ROOT/costa_amd/csrc" "$V/$name/csrc"
for e in "$@"; do
    sed -i "$e" "$V/$name/csrc/tile_kernels.hip" "$V/$name/csrc/engine.hpp"
done
if cmp -s "$ROOT/costa_amd/csrc/tile_kernels.hip" "$V/$name/csrc/tile_kernels.hip" &&
   cmp -s "$ROOT/costa_amd/csrc/engine.hpp" "$V/$name/csrc/engine.hpp"; then
    echo "variant $name: the edits changed nothing" >&2
    exit 1
fi
make -s -C "$V/$name/csrc" -j8 OUT=../lib ../lib/libcosta_amd.so
echo "$V/$name/lib/libcosta_amd.so"
