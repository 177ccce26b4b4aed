#!/bin/bash
# Round 4b: the unchained Cr tile (product) and the unchained + compact-table variant (ucc):
# GPU tests, wrong-launch rates, the golden 4K frame, timing.  Usage: bash tools/gpu_r5j.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
V="$ROOT/jpeg-encoder-and-decoder_amd/lib/variants"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=3 > "$OUT/gpu_tests.txt" 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" "$OUT/gpu_tests.txt" | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/diag_rate.py 60 0 > "$OUT/rate_product.txt" 2>&1 || exit $?
JPGX_LIB=$V/libjpgx_ucc.so timeout -k 10 300 python tools/diag_rate.py 60 0 > "$OUT/rate_ucc.txt" 2>&1 || exit $?
JPGX_LIB=$V/libjpgx_ucc.so timeout -k 10 300 python tools/diag_golden.py 4 > "$OUT/golden_ucc.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/rate_product.txt" "$OUT/rate_ucc.txt"; grep -E "^q" "$OUT/golden_ucc.txt"
ROUNDS=2 bash tools/gpu_r5_price.sh "$1" "chain ucc nox"
