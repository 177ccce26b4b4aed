#!/bin/bash
# Round 5: k_ent_ac with 16 loads per wave (chunks of 512 blocks; variant l16) against the product
# (8 loads, 256 blocks): the entropy GPU tests on both, then batch timing.  Usage: bash tools/gpu_r6au.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_entropy.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ent_tests.txt" 2>&1
rc=$?; tail -2 "$OUT/ent_tests.txt"; [ $rc -eq 0 ] || exit $rc
JPGX_LIB="$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_l16.so" timeout -k 10 300 python -u -m pytest tests/test_entropy.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ent_tests_l16.txt" 2>&1
rc=$?; tail -2 "$OUT/ent_tests_l16.txt"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  EB_MODE=batch timeout -k 10 300 python tools/entropy_bench.py product l16 >> "$OUT/ebench.txt" 2>&1 || { cat "$OUT/ebench.txt"; exit 1; }
done
cat "$OUT/ebench.txt"
