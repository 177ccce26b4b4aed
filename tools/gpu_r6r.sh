#!/bin/bash
# Round 5: PMC counter groups of k_mxs420 in the product and in the build without its exact pass
# (noex420), on the 4:2:0 bench workload.  Usage: bash tools/gpu_r6r.sh OUT
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
OUT="$ROOT/gpurun_out/$1"; mkdir -p "$OUT"
export TMPDIR=/tmp
GROUPS_=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
         "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
         "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ SQ_IFETCH SQ_INSTS_BRANCH SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT")
for name in default noex420; do
  lib=$ROOT/jpeg-encoder-and-decoder_amd/lib/variants/libjpgx_$name.so
  [ "$name" = default ] && lib=$ROOT/jpeg-encoder-and-decoder_amd/lib/libjpgx.so
  i=0
  for grp in "${GROUPS_[@]}"; do
    i=$((i+1)); out=$OUT/$name/g$i; mkdir -p "$out"
    (cd /tmp && JPGX_LIB=$lib timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$out" -o run -- python "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --subsample --sample-ratio 2 --quality 75 > "$out/log" 2>&1); rc=$?
    echo "$name group $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$out/log"; exit $rc; }
  done
done
python tools/pmc_variants_summary.py "$OUT" k_mxs420
