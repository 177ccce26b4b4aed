#!/bin/bash
# Round-4 combined GPU session: the GPU test suite on the product library, error rates of the
# product over many launches (tools/diag_rate.py), and the short-wave kernels against the round-3
# persistent ones (tools/kbench.py).  Every step has its own time limit; a failure ends the script.
# Usage: bash tools/gpu_r4_combo.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT" gpurun_out/r4d
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread --maxfail=3 > "$OUT/gpu_tests.txt" 2>&1
rc=$?; tail -4 "$OUT/gpu_tests.txt"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python tools/diag_rate.py ${RATE_N:-100} 0 1 2 > "$OUT/rate_product.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/rate_product.txt"
KB_SUB=0 timeout -k 10 400 python tools/kbench.py 2 legacy ${KB444:-} > "$OUT/kb444.txt" 2>&1 || exit $?
KB_SUB=1 timeout -k 10 300 python tools/kbench.py 2 l422n > "$OUT/kb422.txt" 2>&1 || exit $?
KB_SUB=2 timeout -k 10 300 python tools/kbench.py 2 l420n > "$OUT/kb420.txt" 2>&1 || exit $?
cat "$OUT/kb444.txt" "$OUT/kb422.txt" "$OUT/kb420.txt"
if [ "${SKEL:-0}" = "1" ]; then
  timeout -k 10 300 ./tools/membench3 r4c > "$OUT/skel_r4c.txt" 2>&1 || exit $?
  cut -c1-150 "$OUT/skel_r4c.txt"
fi
