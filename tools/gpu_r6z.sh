#!/bin/bash
# Round 5: k_mxs / k_mxs422 with 4-6 steps per wave over the three-slot ring (later slots refilled
# by inline-asm LDS-DMA): timing against the product (3 steps), output hash equality, and the
# wrong-launch rate of each variant.  Usage: bash tools/gpu_r6z.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "s4 s5 s6" "s4 s5 s6" || exit $?
for v in s4 s6; do
  JPGX_LIB=jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_$v.so timeout -k 10 300 python tools/diag_rate.py 40 0 1 > "$OUT/rate_$v.txt" 2>&1 || exit $?
  grep -v amdgpu.ids "$OUT/rate_$v.txt"
done
