#!/bin/bash
# Round 5: where k_mxs420's exact-pass time goes (timing-only dissection builds).  Usage: bash tools/gpu_r6q.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
KB_SUB=2 timeout -k 10 500 python tools/kbench.py 3 noex420 e420y e420c e420s1 e420nosingle > "$OUT/kb420.txt" 2>&1 || exit $?
cat "$OUT/kb420.txt"
