#!/bin/bash
# Kernel-trace stats of bench.py for several library variants (GPU box), one rocprofv3 run
# each: per-kernel durations of k_xform and k_fix.  Usage: tools/fix_prof.sh name...
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/fixprof"; mkdir -p "$OUT"
export TMPDIR=/tmp
for v in "$@"; do
  lib="$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_$v.so"
  [ "$v" = default ] && lib="$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx.so"
  (cd /tmp && JPGX_LIB="$lib" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/$v" -o run -- python "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline \
      > "$OUT/$v.json" 2> "$OUT/$v.err") || { echo "$v failed rc=$?"; exit 1; }
  f=$(find "$OUT/$v" -name "*kernel_stats.csv" | head -1)
  echo "== $v: $(grep -o '"ms_per_step": [0-9.]*' "$OUT/$v.json")"
  grep -E "k_xform|k_fix" "$f" | cut -d, -f1-4
done
