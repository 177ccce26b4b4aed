#!/bin/bash
# A/B session: bench.py alternating between the two 4:4:4 kernels (REPS rounds, no CPU leg),
# the true-subsampling benches, then the frames-per-launch sweep of both 4:4:4 kernels.
# Usage (GPU box): bash tools/gpu_ab.sh [REPS]
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/ab"; mkdir -p "$OUT"
export TMPDIR=/tmp
REPS=${1:-3}
summ() { python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_ms'], d['roofline']['frac'], (d.get('output_check') or {}).get('ok'))" "$1"; }
for r in $(seq 1 "$REPS"); do
  for k in xform mx; do
    timeout -k 10 300 python bench.py --kernel $k --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline > "$OUT/bench_${k}_$r.json" 2> "$OUT/bench_${k}_$r.err"; rc=$?
    echo "bench $k rep $r rc=$rc $(summ $OUT/bench_${k}_$r.json)"
    [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${k}_$r.err"; exit $rc; }
  done
done
for v in "1 fused" "1 two-pass" "2 fused" "2 two-pass"; do
  set -- $v
  if [ "$2" = two-pass ]; then export JPGX_LIB="$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx_alt.so"; else unset JPGX_LIB; fi
  timeout -k 10 300 python bench.py --subsample --sample-ratio $1 --quality 75 --steps 20 --warmup 5 --no-cpu-baseline > "$OUT/bench_sr$1_$2.json" 2> "$OUT/bench_sr$1_$2.err"; rc=$?
  echo "bench sr$1 $2 rc=$rc $(summ $OUT/bench_sr$1_$2.json)"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_sr$1_$2.err"; exit $rc; }
done
unset JPGX_LIB
if [ "${SWEEP:-1}" = "1" ]; then
  timeout -k 10 400 python tools/frames_sweep.py "$OUT/frames_sweep.json" xform mx > "$OUT/frames_sweep.log" 2>&1; rc=$?
  echo "sweep rc=$rc"; tail -12 "$OUT/frames_sweep.log"; [ $rc -eq 0 ] || exit $rc
fi
