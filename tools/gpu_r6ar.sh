#!/bin/bash
# Round 5: k_mxs with an XCD-contiguous workgroup mapping (variant xcd: workgroup b runs the
# range of (b % 8) * (G / 8) + b / 8, so each XCD streams one contiguous eighth) against the product.
# Usage: bash tools/gpu_r6ar.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "xcd"
