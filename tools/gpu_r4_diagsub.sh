#!/bin/bash
# Round-4 diagnostics (GPU box): tools/diag_sub.py over the product and variant libraries.
# Usage: bash tools/gpu_r4_diagsub.sh REPS "SRS" lib...
set -u
mkdir -p gpurun_out/r4d
export TMPDIR=/tmp
V=jpeg-encoder-and-decoder_amd/lib/variants
R=$1; SRS=$2; shift 2
for v in "$@"; do
  lib=$PWD/$V/libjpgx_$v.so; [ "$v" = product ] && lib=$PWD/jpeg-encoder-and-decoder_amd/lib/libjpgx.so
  JPGX_LIB=$lib timeout -k 10 300 python tools/diag_sub.py $R $SRS > gpurun_out/r4d/s_$v.txt 2>&1 || exit $?
  echo "== $v"; grep "rep" gpurun_out/r4d/s_$v.txt | cut -c1-150
done
