#!/bin/bash
# Round-4 diagnostics (GPU box): the golden 4K frame through the product and variant libraries
# (tools/diag_golden.py), mismatches per launch.  Usage: bash tools/gpu_r4_diag.sh REPS lib...
set -u
mkdir -p gpurun_out/r4d
export TMPDIR=/tmp
V=jpeg-encoder-and-decoder_amd/lib/variants
R=$1; shift
for v in "$@"; do
  lib=$PWD/$V/libjpgx_$v.so; [ "$v" = product ] && lib=$PWD/jpeg-encoder-and-decoder_amd/lib/libjpgx.so
  JPGX_LIB=$lib timeout -k 10 300 python tools/diag_golden.py $R > gpurun_out/r4d/$v.txt 2>&1 || exit $?
  echo "== $v"; grep "rep" gpurun_out/r4d/$v.txt | awk '{print $1, $2, $3, $4, $5, $6, $7, $8}' | tr '\n' ';'; echo
done
