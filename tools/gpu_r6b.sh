#!/bin/bash
# Round 5 fault probe: the dumped R / scale values of k_mxs across launches (tools/diag_dump.py) in
# the padded and unpadded B-from-global reproducers.  Usage: bash tools/gpu_r6b.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
V="$ROOT/jpeg-encoder-and-decoder_amd/lib/variants"
export TMPDIR=/tmp
for v in ${VARS:-dump dump0}; do
  JPGX_LIB=$V/libjpgx_$v.so timeout -k 10 300 python tools/${DIAG:-diag_dump.py} ${N:-5} > "$OUT/dump_$v.txt" 2>&1 || exit $?
  grep -v amdgpu.ids "$OUT/dump_$v.txt"
done
