#!/bin/bash
# Round 4b: GPU tests, wrong-launch rates (tools/diag_rate.py, every sample ratio) and the timing
# A/B against the round-4 exact pass (variant r4) and the no-exact probe.  Usage: bash tools/gpu_r5g.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=3 > "$OUT/gpu_tests.txt" 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" "$OUT/gpu_tests.txt" | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/diag_rate.py ${RATE_N:-60} 0 1 2 > "$OUT/rate_product.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/rate_product.txt"
ROUNDS=2 bash tools/gpu_r5_price.sh "$1" "${KB444:-head nox}" ${KB422:-head} ${KB420:-head}
