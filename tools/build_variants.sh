#!/bin/bash
# Build tuning variants of libjpgx.so (same sources, different compile-time knobs) into
# jpeg-encoder-and-decoder_amd/lib/variants/.  Usage: [MX_SRC=patched jpgx_mx.hip] tools/build_variants.sh name "FLAGS" ...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PKG=$ROOT/jpeg-encoder-and-decoder_amd
OUT=$PKG/lib/variants
mkdir -p "$OUT" "$PKG/build/variants"
make -s -C "$PKG" >/dev/null
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  obj=$PKG/build/variants/$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-slp-vectorize -I"$ROOT/include" \
      $flags -c "$PKG/csrc/jpgx_kernels.hip" -o "$obj"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-slp-vectorize -I"$ROOT/include" \
      $flags -c "${MX_SRC:-$PKG/csrc/jpgx_mx.hip}" -o "$PKG/build/variants/${name}_mx.o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -fno-slp-vectorize -I"$ROOT/include" \
      $flags -c "$PKG/csrc/jpgx_entropy.hip" -o "$PKG/build/variants/${name}_ent.o"
  g++ -O2 -fPIC -std=c++17 -ffp-contract=off -I"$ROOT/include" $flags \
      -c "$PKG/csrc/jpgx_plan.cpp" -o "$PKG/build/variants/${name}_plan.o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT/libjpgx_$name.so" "$obj" "$PKG/build/variants/${name}_mx.o" \
      "$PKG/build/variants/${name}_plan.o" "$PKG"/build/jpgx_block.o "$PKG"/build/jpgx_jpgdata.o \
      "$PKG"/build/jpgx_jfif.o "$PKG/build/variants/${name}_ent.o" "$PKG"/build/jpgx_host.o -lpthread
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -I"$ROOT/include" \
      $flags --cuda-device-only -S "${MX_SRC:-$PKG/csrc/jpgx_mx.hip}" -o "$PKG/build/variants/$name.s"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize -I"$ROOT/include" \
      $flags --cuda-device-only -S "$PKG/csrc/jpgx_kernels.hip" -o "$PKG/build/variants/${name}_k.s"

  echo "$name (k_mx): $(grep -E '^\s+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count):' "$PKG/build/variants/$name.s" | head -3 | tr -s ' ' | tr '\n' ' ')"
done
