#!/bin/bash
# Round 5 fault probes: wrong-launch rates (tools/diag_rate.py, 20 x 2 x 4K q75, 4:4:4) of the
# B-from-global (bgl*) and one-wave-workgroup (w1*) reproducers with padding after each product
# group (pad) or every A operand kept live to the step's end (keep).  Usage: bash tools/gpu_r6a.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
V="$ROOT/jpeg-encoder-and-decoder_amd/lib/variants"
export TMPDIR=/tmp
for v in ${VARS:-bgl bglpad bglkeep w1 w1pad w1keep}; do
  JPGX_LIB=$V/libjpgx_$v.so timeout -k 10 200 python tools/diag_rate.py ${N:-20} 0 > "$OUT/rate_$v.txt" 2>&1 || exit $?
  grep -v amdgpu.ids "$OUT/rate_$v.txt"
done
