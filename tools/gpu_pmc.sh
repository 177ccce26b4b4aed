#!/bin/bash
# PMC passes over a short bench run, one counter group per rocprofv3 run (kernel trace only).
# Usage: tools/gpu_pmc.sh OUTDIR "GROUP1" "GROUP2" ...   (run on the GPU box)
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$1"; shift; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$OUT/p$i.log" 2>&1; rc=$?
  echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
