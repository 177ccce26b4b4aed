#!/bin/bash
# Variant timing session: GPU parity tests (default library), then tools/variant_bench.py.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -15 "$OUT/pytest_gpu.log"
  if [ $rc -ne 0 ]; then exit $rc; fi
fi
timeout -k 10 600 python tools/variant_bench.py "$@" > "$OUT/variants.log" 2>&1; rc=$?
cat "$OUT/variants.log"; exit $rc
