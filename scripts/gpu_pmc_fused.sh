#!/bin/bash
# PMC passes over the default fused FD4 step and the WENO5 stage (kernel-trace only).
set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/pmc
PMC_SETS_OVERRIDE='"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"' \
PMC_JOBS="${PMC_JOBS:-fused:ADVDIFF_STEP_EDGE=1 fused:ADVDIFF_STEP_EDGE=0}" bash scripts/pmc_run.sh && \
python3 bench/summarize_pmc.py gpurun_out/pmc > gpurun_out/pmc_summary.md
