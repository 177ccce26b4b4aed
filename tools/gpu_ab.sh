#!/bin/bash
# A/B session: GPU parity tests on the default kernel, then bench default vs JPGX_KERNEL=xform.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -30 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in default xform; do
  if [ $k = xform ]; then export JPGX_KERNEL=xform; else unset JPGX_KERNEL; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_$k.json" 2> "$OUT/bench_$k.err"; rc=$?
  echo "bench $k rc=$rc"; cat "$OUT/bench_$k.json"; tail -3 "$OUT/bench_$k.err"; [ $rc -eq 0 ] || exit $rc
done
