#!/bin/bash
# Round 5: what the whole-wave exact path's latency is made of (timing-only builds: no division,
# no cross-lane sum, no pixel reads) against the product and the no-exact build.  Usage: bash tools/gpu_r6v.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
ROUNDS=3 bash tools/gpu_r5_price.sh "$1" "noex444b xnodiv xnored xnopix" || exit $?
