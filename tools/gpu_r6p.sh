#!/bin/bash
# Round 5: the product after the B-operand reload and without the exact pass's lgkmcnt(0): GPU
# tests, wrong-launch rates, golden frames, timing against the r6m build.  Usage: bash tools/gpu_r6p.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=3 > "$OUT/gpu_tests.txt" 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" "$OUT/gpu_tests.txt" | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/diag_rate.py ${N:-100} 0 1 2 > "$OUT/rate_product.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/rate_product.txt"
timeout -k 10 300 python tools/diag_golden.py 8 > "$OUT/golden_product.txt" 2>&1 || exit $?
grep -E "^q" "$OUT/golden_product.txt" | sort | uniq -c | head -4
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "r5b" || exit $?
