#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel trace.
# Every GPU step has its own time limit; a crash/timeout ends the script (no retries).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-20}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --maxfail=5 > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -25 "$OUT/pytest_gpu.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 "$OUT/smoke.log"; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python bench.py --steps $STEPS --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"; rc=$?
echo "bench rc=$rc"; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"; [ $rc -eq 0 ] || exit $rc
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python "$ROOT/bench.py" --steps $STEPS --warmup 5 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"; rc=$?
  echo "rocprof rc=$rc"; find "$OUT/prof" -name "*stats*" | head; [ $rc -eq 0 ] || exit $rc
fi
