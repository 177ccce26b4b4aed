#!/bin/bash
# Round 5: the product with 16 loads per wave in k_ent_ac: entropy + config-scale GPU tests, batch
# timing and rocprofv3 --stats (tools/gpu_r6ao.sh).  Usage: bash tools/gpu_r6av.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_r6ao.sh "$1"
