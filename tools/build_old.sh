#!/bin/bash
# Build lib/variants/libjpgx_<name>.so from the product sources with csrc/<file> in place of
# csrc/jpgx_mx.hip (A/B of a previous k_mx on the same box).  Usage: tools/build_old.sh name file
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/jpeg-encoder-and-decoder_amd
name=$1; file=$2
mkdir -p "$PKG/lib/variants" "$PKG/build/variants"
make -s -C "$PKG" >/dev/null
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-slp-vectorize -I"$ROOT/include" \
    -c "$PKG/csrc/$file" -o "$PKG/build/variants/${name}_mx.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$PKG/lib/variants/libjpgx_$name.so" \
    "$PKG/build/jpgx_kernels.o" "$PKG/build/variants/${name}_mx.o" "$PKG/build/jpgx_plan.o" \
    "$PKG"/build/jpgx_block.o "$PKG"/build/jpgx_jpgdata.o "$PKG"/build/jpgx_jfif.o \
    "$PKG"/build/jpgx_entropy.o "$PKG"/build/jpgx_host.o -lpthread
echo "built lib/variants/libjpgx_$name.so"
