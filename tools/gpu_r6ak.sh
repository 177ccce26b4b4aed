#!/bin/bash
# Round 5: the batched entropy statistics: GPU tests, per-frame and batch timing, rocprofv3
# --stats of the batch bench.  Usage: bash tools/gpu_r6ak.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_entropy.py tests/test_config_scale.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/ent_tests.txt" 2>&1
rc=$?; tail -3 "$OUT/ent_tests.txt"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  EB_MODE=frame timeout -k 10 300 python tools/entropy_bench.py >> "$OUT/ebench.txt" 2>&1 || { cat "$OUT/ebench.txt"; exit 1; }
  EB_MODE=batch timeout -k 10 300 python tools/entropy_bench.py >> "$OUT/ebench.txt" 2>&1 || { cat "$OUT/ebench.txt"; exit 1; }
done
cat "$OUT/ebench.txt"
cd /tmp && EB_MODE=batch timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$ROOT/tools/entropy_bench.py" > "$OUT/prof.log" 2>&1 || { tail -20 "$OUT/prof.log"; exit 1; }
find "$OUT/prof" -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -6
