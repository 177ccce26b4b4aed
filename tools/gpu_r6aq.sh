#!/bin/bash
# Round 5: wrong-launch rate of the committed product at N (default 20,000) launches per sample ratio
# (tools/diag_rate.py: 2 x 4K q75 per launch, every block against the oracle on the GPU).
# Usage: bash tools/gpu_r6aq.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u tools/diag_rate.py ${N:-20000} 0 1 2 > "$OUT/rate.txt" 2>&1; rc=$?
grep -v amdgpu.ids "$OUT/rate.txt"; exit $rc
