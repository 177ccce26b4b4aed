#!/bin/bash
# Round-4 session (GPU box): GPU tests on the product library, then the short-wave 4:2:2 / 4:2:0
# kernels against the persistent ones (tools/kbench.py, KB_SUB), then the skeleton's occupancy /
# MFMA sweep (membench3 r4c).  Usage: bash tools/gpu_r4_sub.sh OUTDIR [TESTS=1] [SKEL=1]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -eq 0 ] || exit $rc
fi
KB_SUB=0 timeout -k 10 300 python tools/kbench.py 2 nokc w1c3 legacy > "$OUT/kb444.txt" 2>&1 || exit $?
KB_SUB=1 timeout -k 10 300 python tools/kbench.py 2 l422 s422w4 > "$OUT/kb422.txt" 2>&1 || exit $?
KB_SUB=2 timeout -k 10 300 python tools/kbench.py 2 l420 s420w4 > "$OUT/kb420.txt" 2>&1 || exit $?
cat "$OUT/kb444.txt" "$OUT/kb422.txt" "$OUT/kb420.txt"
if [ "${SKEL:-1}" = "1" ]; then
  timeout -k 10 300 ./tools/membench3 r4c > "$OUT/skel_r4c.txt" 2>&1 || exit $?
  cut -c1-140 "$OUT/skel_r4c.txt"
fi
