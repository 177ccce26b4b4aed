#!/bin/bash
# Round 5: k_mxs's sensitivity to its workgroup image (timing probes: noextab drops the exact pass's
# 1.8 KiB of tables from the image -- not exact; padimg adds 1 KiB; bglob reads the B operands from
# global memory at the wave's top instead, the image shrinking by 4 KiB -- exact, rate checked).
# Usage: bash tools/gpu_r6aa.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "noextab bglob slimprobe" || exit $?


