#!/bin/bash
# True-subsampling session: GPU subsample tests, then bench.py --subsample for 4:2:2 (fused and
# two-pass) and 4:2:0.  Usage (GPU box): bash tools/gpu_sub.sh
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/sub"; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_subsample.py tests/test_bench_gpu.py -m gpu -v --timeout 200 --timeout-method thread --maxfail=3 > "$OUT/pytest.log" 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|passed|failed|Error" "$OUT/pytest.log" | tail -15
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in "1 fused" "1 two-pass" "2 two-pass"; do
  set -- $v
  if [ "$2" = two-pass ]; then export JPGX_LIB="$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx_alt.so"; else unset JPGX_LIB; fi
  timeout -k 10 300 python bench.py --subsample --sample-ratio $1 --quality 75 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_sr$1_$2.json" 2> "$OUT/bench_sr$1_$2.err"; rc=$?
  echo "bench sr$1 $2 rc=$rc $(cat $OUT/bench_sr$1_$2.json)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_sr$1_$2.err"; exit $rc; }
done
