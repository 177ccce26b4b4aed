#!/bin/bash
# Round 5: A/B of the next k_mxs / k_mxs420 candidates against the product, and the wrong-launch
# rates of the two that break the round-4 chained-product rule (crchain, nof420) -- a direct test of
# that rule now that packed fp32 is gone.  Usage: bash tools/gpu_r6n.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
V=jpeg-encoder-and-decoder_amd/lib/variants
JPGX_LIB=$V/libjpgx_crchain.so timeout -k 10 300 python tools/diag_rate.py 60 0 > "$OUT/rate_crchain.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/rate_crchain.txt"
JPGX_LIB=$V/libjpgx_nof420.so timeout -k 10 300 python tools/diag_rate.py 60 2 > "$OUT/rate_nof420.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/rate_nof420.txt"
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "nolgkm crchain noex444" "noex422" "nof420 noex420" || exit $?
