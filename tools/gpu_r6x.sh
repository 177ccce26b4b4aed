#!/bin/bash
# Round 5: k_mxs420 with two step pairs per wave (variant p2): 4:2:0 GPU tests and wrong-launch
# rate on the variant library, then timing against the product.  Usage: bash tools/gpu_r6x.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
V=jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_p2.so
JPGX_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_subsample.py -m gpu -q --timeout 120 --timeout-method thread --maxfail=3 > "$OUT/p2_tests.txt" 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" "$OUT/p2_tests.txt" | tail -8; [ $rc -eq 0 ] || [ $rc -eq 5 ] || exit $rc
JPGX_LIB=$V timeout -k 10 300 python tools/diag_rate.py 60 2 > "$OUT/rate_p2.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/rate_p2.txt"
KB_SUB=2 timeout -k 10 400 python tools/kbench.py 3 r5a p2 > "$OUT/kb420.txt" 2>&1 || exit $?
cat "$OUT/kb420.txt"
