#!/bin/bash
# Round 5: validation of the scalar column pass (no packed fp32 in the MFMA kernels): GPU tests,
# wrong-launch rates in every mode, the golden 4K frame, timing against the packed build (pkd),
# and the packed-form probe.  Usage: bash tools/gpu_r6m.sh OUT
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
grep -E "^q" "$OUT/golden_product.txt"
ROUNDS=${ROUNDS:-3} bash tools/gpu_r5_price.sh "$1" "${VARS444:-pkd}" "${VARS422:-pkd}" "${VARS420:-pkd}" || exit $?
timeout -k 10 250 ./tools/probes/pk_hazard5 8192 400 1 > "$OUT/pk_hazard5_set1.txt" 2>&1 || exit $?
cat "$OUT/pk_hazard5_set1.txt"
timeout -k 10 250 ./tools/probes/pk_hazard5 8192 400 2 > "$OUT/pk_hazard5_set2.txt" 2>&1 || exit $?
cat "$OUT/pk_hazard5_set2.txt"
