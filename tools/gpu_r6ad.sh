#!/bin/bash
# Round 5: s_setprio variants against the product.  k_mxs only: prio1 (prologue at priority 3),
# prio2 (priority 1 until the last step), prio3 (the stores at priority 2); all three kernels:
# pall3 / pall1 (prologue -- image and pixel DMA issue -- at priority 3 / 1).
# Usage: bash tools/gpu_r6ad.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "prio1 prio2 prio3 pall3 pall1" "pall3 pall1" "pall3 pall1"
