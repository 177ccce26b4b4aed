#!/bin/bash
# Round-4 (GPU box): kernel stats and PMC passes of the true 4:2:2 / 4:2:0 bench (k_mxs422 / k_mxs420),
# one counter group per rocprofv3 run (kernel trace only).  Output: gpurun_out/r4sub/
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
OUT="$ROOT/gpurun_out/${1:-r4sub}"; mkdir -p "$OUT"
cd /tmp
for sr in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/stats$sr" -o run -- python "$ROOT/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --subsample --sample-ratio $sr --quality 75 > "$OUT/bench$sr.json" 2> "$OUT/bench$sr.err" || exit $?
  echo "sr$sr stats ok"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"; do
    i=$((i+1))
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/sr${sr}_p$i" -o run -- python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --subsample --sample-ratio $sr --quality 75 > "$OUT/sr${sr}_p$i.log" 2>&1 || exit $?
    echo "sr$sr pmc pass $i ok"
  done
done
