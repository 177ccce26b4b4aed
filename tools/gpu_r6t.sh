#!/bin/bash
# Round 5: prefilter rates (counting build cnt2) and the no-exact builds that keep every flag bit
# live (noex420b / noex444b).  Usage: bash tools/gpu_r6t.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
JPGX_LIB=jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_cnt3.so timeout -k 10 300 python tools/diag_exact_time.py 10 > "$OUT/prefilter_count.txt" 2>&1 || exit $?
grep -v amdgpu.ids "$OUT/prefilter_count.txt"
true
