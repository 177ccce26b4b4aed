#!/bin/bash
# Round-4 A/B session (GPU box): the GPU test suite on the product library, then bench.py
# (fresh input, settled, output checked against the goldens) on each variant library,
# interleaved rounds.  Usage: bash tools/gpu_r4_ab.sh OUTDIR "variant ..." [ROUNDS] [TESTS=1]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
VARS=$2; ROUNDS=${3:-2}
export TMPDIR=/tmp
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/gpu_tests.txt" 2>&1
  rc=$?; tail -3 "$OUT/gpu_tests.txt"; [ $rc -eq 0 ] || exit $rc
fi
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(d['value'], r['kernel_ms'], r['frac'], (d.get('output_check') or {}).get('ok'))" "$1"; }
for r in $(seq 1 "$ROUNDS"); do
  for v in $VARS; do
    lib="$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_$v.so"
    [ "$v" = product ] && lib="$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx.so"
    JPGX_LIB=$lib timeout -k 10 200 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline $BENCH_ARGS > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err"; rc=$?
    echo "bench $v round $r rc=$rc $(summ $OUT/bench_${v}_$r.json)"
    [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${v}_$r.err"; exit $rc; }
  done
done
