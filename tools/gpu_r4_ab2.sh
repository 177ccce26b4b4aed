#!/bin/bash
# Round-4 A/B (GPU box): wrong-launch rates of variant libraries (tools/diag_rate.py), then
# tools/kbench.py product vs the variants for 4:4:4, 4:2:2 and 4:2:0.  Usage: bash tools/gpu_r4_ab2.sh OUT lib...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; shift; mkdir -p "$OUT"
export TMPDIR=/tmp
V=jpeg-encoder-and-decoder_amd/lib/variants
for v in "$@"; do
  JPGX_LIB=$PWD/$V/libjpgx_$v.so timeout -k 10 300 python tools/diag_rate.py ${RATE_N:-60} 0 1 2 > "$OUT/rate_$v.txt" 2>&1 || exit $?
  grep -v amdgpu.ids "$OUT/rate_$v.txt"
done
for sr in 0 1 2; do
  KB_SUB=$sr timeout -k 10 400 python tools/kbench.py 2 "$@" > "$OUT/kb$sr.txt" 2>&1 || exit $?
  echo "== sr$sr"; cat "$OUT/kb$sr.txt"
done
