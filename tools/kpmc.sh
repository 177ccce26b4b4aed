#!/bin/bash
# PMC counters of kbench's workload per library, one rocprofv3 run per (library, counter group),
# kernel trace only.  Usage (GPU box): tools/kpmc.sh OUTDIR "COUNTERS" name ... ; then
# python tools/kpmc_summary.py gpurun_out/OUTDIR KERNEL.  KB_SUB selects the mode as in kbench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$1"; C=$2; shift 2
mkdir -p "$OUT"; export TMPDIR=/tmp
for n in "$@"; do
  if [ "$n" = product ]; then lib=$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx.so
  else lib=$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_$n.so; fi
  tag=$n-$(echo "$C" | tr ' ' '+' | cut -c1-40)
  (cd /tmp && JPGX_LIB=$lib KB_REPS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv \
      -d "$OUT/$tag" -o run -- python "$ROOT/tools/kbench_child.py" > "$OUT/$tag.log" 2>&1); rc=$?
  echo "kpmc $tag rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$tag.log"; exit $rc; }
done
