#!/bin/bash
# Round 4b: validation of the product with the exact pass's tables in LDS (GPU tests, wrong-launch
# rates in every mode, the golden 4K frame) and its timing against the previous product (r5head).
# Usage: bash tools/gpu_r5m.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=3 > "$OUT/gpu_tests.txt" 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" "$OUT/gpu_tests.txt" | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/diag_rate.py 100 0 1 2 > "$OUT/rate_product.txt" 2>&1 || exit $?
timeout -k 10 300 python tools/diag_golden.py 8 > "$OUT/golden_product.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/rate_product.txt"; grep -E "^q" "$OUT/golden_product.txt"
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "r5head"
