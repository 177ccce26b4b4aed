#!/bin/bash
# Round-4 diagnostics (GPU box): tools/diag_rate.py over the product and variant libraries.
# Usage: bash tools/gpu_r4_rate.sh N "SRS" lib...
set -u
mkdir -p gpurun_out/r4d
export TMPDIR=/tmp
V=jpeg-encoder-and-decoder_amd/lib/variants
N=$1; SRS=$2; shift 2
for v in "$@" ${RATE_EXTRA-gap15 gap15nk}; do
  lib=$PWD/$V/libjpgx_$v.so; [ "$v" = product ] && lib=$PWD/jpeg-encoder-and-decoder_amd/lib/libjpgx.so
  JPGX_LIB=$lib timeout -k 10 300 python tools/diag_rate.py $N $SRS > gpurun_out/r4d/r_$v.txt 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r4d/r_$v.txt
done
