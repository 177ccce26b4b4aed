#!/bin/bash
# Timing-only A/B of variant libraries against the product (tools/kbench.py), 4:4:4 and optionally
# 4:2:x.  Usage: bash tools/gpu_r5_price.sh OUT "444 variants" ["422 variants"] ["420 variants"]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
KB_SUB=0 timeout -k 10 400 python tools/kbench.py ${ROUNDS:-2} $2 > "$OUT/kb444.txt" 2>&1 || exit $?
cat "$OUT/kb444.txt"
if [ -n "${3:-}" ]; then
  KB_SUB=1 timeout -k 10 300 python tools/kbench.py ${ROUNDS:-2} $3 > "$OUT/kb422.txt" 2>&1 || exit $?
  cat "$OUT/kb422.txt"
fi
if [ -n "${4:-}" ]; then
  KB_SUB=2 timeout -k 10 300 python tools/kbench.py ${ROUNDS:-2} $4 > "$OUT/kb420.txt" 2>&1 || exit $?
  cat "$OUT/kb420.txt"
fi
