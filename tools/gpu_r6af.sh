#!/bin/bash
# Round 5: cache policy of the pixel LDS-DMA (nt / sc1 / sc0 sc1 nt; default in the product)
# against the product, every kernel.  Usage: bash tools/gpu_r6af.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "ldnt ldsc1 ldsc01nt" "ldnt ldsc1 ldsc01nt" "ldnt ldsc1 ldsc01nt"
