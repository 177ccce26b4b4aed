#!/bin/bash
# GPU parity tests of the current sources, then the fresh-input bench of the current library
# against lib/variants/libjpgx_prev.so (tools/build_old.sh prev <file>) on the same box:
# 4:4:4 q90 (REPS rounds), true 4:2:2 and 4:2:0 q75 (one round each).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
REPS=${REPS:-2} bash tools/gpu_libs_bench.sh default prev || exit $?
[ "${SUB:-1}" = "1" ] || exit 0
REPS=1 BENCH_ARGS="--subsample --sample-ratio 1 --quality 75" bash tools/gpu_libs_bench.sh default prev || exit $?
REPS=1 BENCH_ARGS="--subsample --sample-ratio 2 --quality 75" bash tools/gpu_libs_bench.sh default prev || exit $?
