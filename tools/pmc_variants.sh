#!/bin/bash
# PMC counter groups (one rocprofv3 run each, kernel trace only) over a short bench.py run, for
# each named library variant (lib/variants/libjpgx_<name>.so; "default" = lib/libjpgx.so).
# Usage (GPU box): tools/pmc_variants.sh name1 name2 ...   -> gpurun_out/pmcv/<name>/g<i>/
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR")
for name in "$@"; do
  lib=$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_$name.so
  [ "$name" = default ] && lib=$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx.so
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1)); out=$ROOT/gpurun_out/pmcv/$name/g$i; mkdir -p "$out"
    (cd /tmp && JPGX_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$out" -o run -- python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$out/log" 2>&1); rc=$?
    echo "$name group $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/log"; exit $rc; }
  done
done
