#!/bin/bash
# GPU parity tests, then repeated whole-frame golden checks of the current library and of
# lib/variants/libjpgx_prev.so (the build before the MFMA operand rule), then the A/B bench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1; rc=$?
echo "pytest rc=$rc"; tail -4 "$OUT/pytest_gpu.log"
[ $rc -eq 0 ] || exit $rc
echo "== current"; timeout -k 10 300 python -u tools/stress_golden.py ${REPS_STRESS:-3}; echo "rc=$?"
[ "${STRESS_PREV:-0}" = "1" ] && { echo "== prev"; JPGX_LIB=$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_prev.so timeout -k 10 300 python -u tools/stress_golden.py ${REPS_STRESS:-3}; echo "rc=$?"; }
REPS=2 bash tools/gpu_libs_bench.sh default prev || exit $?
REPS=1 BENCH_ARGS="--subsample --sample-ratio 1 --quality 75" bash tools/gpu_libs_bench.sh default prev || exit $?
REPS=1 BENCH_ARGS="--subsample --sample-ratio 2 --quality 75" bash tools/gpu_libs_bench.sh default prev || exit $?
