#!/bin/bash
# Round 4b diagnostics: wrong-launch rates of the divisors-in-LDS (qlds) and padded-image (pad)
# variants of k_mxs.  Usage: bash tools/gpu_r5k.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
V="$ROOT/jpeg-encoder-and-decoder_amd/lib/variants"
export TMPDIR=/tmp
for v in ${VARS:-qlds pad}; do
  JPGX_LIB=$V/libjpgx_$v.so timeout -k 10 300 python tools/diag_rate.py 80 0 > "$OUT/rate_$v.txt" 2>&1 || exit $?
  JPGX_LIB=$V/libjpgx_$v.so timeout -k 10 300 python tools/diag_golden.py 4 > "$OUT/golden_$v.txt" 2>&1 || exit $?
done
grep -v amdgpu.ids "$OUT"/rate_*.txt; grep -E "^lib|^q" "$OUT"/golden_*.txt
