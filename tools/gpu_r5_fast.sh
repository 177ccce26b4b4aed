#!/bin/bash
# Round 4b: GPU tests on the product, then timing A/Bs (tools/gpu_r5_price.sh).
# Usage: bash tools/gpu_r5_fast.sh OUT "444 variants" ["422 variants"] ["420 variants"]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=3 > "$OUT/gpu_tests.txt" 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" "$OUT/gpu_tests.txt" | tail -8; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r5_price.sh "$@"
