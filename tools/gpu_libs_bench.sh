#!/bin/bash
# bench.py (fresh input, settled, output checked against the goldens) over variant libraries,
# interleaved rounds.  Usage (GPU box): REPS=2 bash tools/gpu_libs_bench.sh default mxg2 ...
# ("default" = lib/libjpgx.so; NAME = lib/variants/libjpgx_NAME.so)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/libs"; mkdir -p "$OUT"
export TMPDIR=/tmp
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['roofline']['frac'], (d.get('output_check') or {}).get('ok'))" "$1"; }
for r in $(seq 1 "${REPS:-2}"); do
  for n in "$@"; do
    if [ "$n" = default ]; then lib=$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx.so
    else lib=$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_$n.so; fi
    JPGX_LIB=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} \
      > "$OUT/bench_${n}_$r.json" 2> "$OUT/bench_${n}_$r.err"; rc=$?
    echo "bench $n rep $r rc=$rc $(summ $OUT/bench_${n}_$r.json)"
    # rc 3 = output differs from the goldens (accepted for timing-only builds with ALLOW_WRONG=1)
    if [ $rc -eq 3 ] && [ "${ALLOW_WRONG:-0}" = "1" ]; then continue; fi
    [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${n}_$r.err"; exit $rc; }
  done
done
