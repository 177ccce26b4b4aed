#!/bin/bash
# Round 5: entropy-statistics variants (tools/entropy_bench.py): 16-bit packed vs 32-bit LDS
# counters, ds_bpermute vs DPP block scan.  Usage: bash tools/gpu_r6aj.sh OUT VARIANTS...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; shift; mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 300 python tools/entropy_bench.py product "$@" >> "$OUT/ebench.txt" 2>&1 || { cat "$OUT/ebench.txt"; exit 1; }
done
cat "$OUT/ebench.txt"
