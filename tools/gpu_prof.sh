#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, kernel trace only) over a short bench.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/pmc"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
ARGS="--steps ${STEPS:-5} --warmup 2 --no-cpu-baseline"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python "$ROOT/bench.py" $ARGS > "$OUT/p$i.log" 2>&1; rc=$?
  echo "pmc pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/p$i.log"; exit $rc; }
done
