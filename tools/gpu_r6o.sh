#!/bin/bash
# Round 5: exact-pass counts per kernel on the bench workload (counting build).  Usage: bash tools/gpu_r6o.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
JPGX_LIB=jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_cnt.so timeout -k 10 300 python tools/diag_exact_count.py 10 > "$OUT/exact_count.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/exact_count.txt"
