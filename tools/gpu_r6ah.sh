#!/bin/bash
# Round 5: the two-kernel entropy statistics: their GPU tests, then tools/gpu_r6ag.sh (timing and
# rocprofv3 --stats).  Usage: bash tools/gpu_r6ah.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_entropy.py tests/test_config_scale.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ent_tests.txt" 2>&1
rc=$?; tail -5 "$OUT/ent_tests.txt"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r6ag.sh "$1"
