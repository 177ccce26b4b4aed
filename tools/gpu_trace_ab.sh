#!/bin/bash
# Per-launch kernel durations over a long back-to-back run, k_xform vs k_mx (power/clock drift).
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for k in xform mx; do
  if [ "$k" = xform ]; then export JPGX_LIB="$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx_alt.so"; else unset JPGX_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$ROOT/gpurun_out/trace_$k" -o run -- python "$ROOT/bench.py" --steps ${STEPS:-80} --warmup 5 --no-cpu-baseline > "$ROOT/gpurun_out/trace_$k.json" 2>&1; rc=$?
  echo "$k rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
