#!/bin/bash
# Round measurement session on ONE GPU box: parity tests, smoke, bench (with the CPU leg),
# rocprofv3 kernel stats of the same bench command, then the PMC passes (one counter group per
# rocprofv3 run, kernel trace only) -- tools/pmc_summary.py turns gpurun_out/ into the
# committed profile.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_check.sh || exit $?
bash tools/gpu_pmc.sh pmc "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum" \
  "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES" || exit $?
