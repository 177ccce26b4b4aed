#!/bin/bash
# Round 5: k_mxs with interleaved steps (variant ilv: wave w of a workgroup computes steps w, w + 4,
# w + 8 of the workgroup's 12, so the four waves' concurrent stores are contiguous) against the
# product.  Usage: bash tools/gpu_r6as.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "ilv"
