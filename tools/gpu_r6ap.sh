#!/bin/bash
# Round 5: k_ent_ac with a dense-lane fast path (variant "dense") against the product: the entropy
# GPU tests run against the variant library, then batch timing.  Usage: bash tools/gpu_r6ap.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
JPGX_LIB="$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_dense.so" timeout -k 10 300 python -u -m pytest tests/test_entropy.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ent_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/ent_tests.txt"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  EB_MODE=batch timeout -k 10 300 python tools/entropy_bench.py product dense >> "$OUT/ebench.txt" 2>&1 || { cat "$OUT/ebench.txt"; exit 1; }
done
cat "$OUT/ebench.txt"
