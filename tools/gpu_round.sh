#!/bin/bash
# Round-end measurement session on the GPU box: parity tests, smoke, bench, rocprofv3 kernel
# stats, and the FETCH_SIZE / WRITE_SIZE PMC passes (one counter per run) for the traffic figure.
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash tools/gpu_check.sh || exit $?
bash tools/gpu_pmc.sh pmc "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum" || exit $?
