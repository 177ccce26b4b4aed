#!/bin/bash
# Round 5: bench.py with the repeated-launch output check: its GPU tests, the default bench line,
# and the true 4:2:0 line.  Usage: bash tools/gpu_r6ae.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_bench_gpu.py -m gpu -q --timeout 300 --timeout-method thread > "$OUT/bench_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/bench_tests.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
cat "$OUT/bench.json"
timeout -k 10 300 python bench.py --subsample --sample-ratio 2 --quality 75 --no-cpu-baseline > "$OUT/bench420.json" 2> "$OUT/bench420.err" || exit $?
cat "$OUT/bench420.json"
