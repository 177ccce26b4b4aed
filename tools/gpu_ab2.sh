#!/bin/bash
# GPU tests (parity) then an interleaved bench A/B of the product library against variants.
# Usage (GPU box): bash tools/gpu_ab2.sh variant...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
  [ $rc -eq 0 ] || exit $rc
fi
REPS=${REPS:-3} bash tools/gpu_libs_bench.sh default "$@"
