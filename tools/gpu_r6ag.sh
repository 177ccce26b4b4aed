#!/bin/bash
# Round 5: the entropy-stage statistics timed (tools/entropy_bench.py) and their kernels'
# rocprofv3 --stats.  Usage: bash tools/gpu_r6ag.sh OUT [LIB ...]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; shift; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python tools/entropy_bench.py "$@" > "$OUT/ebench.txt" 2>&1 || { cat "$OUT/ebench.txt"; exit 1; }
cat "$OUT/ebench.txt"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/tools/entropy_bench.py" > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-250
