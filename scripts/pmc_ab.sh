#!/bin/bash
# PMC passes (kernel-trace only) of one profile target under several kernel variants:
#   PMC_TARGET=fused PMC_CFGS="0 21" bash scripts/pmc_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE")
for cfg in ${PMC_CFGS:-0}; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    ADVDIFF_STEP_CFG=$cfg timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv \
      -d gpurun_out/pmc/${PMC_TARGET:-fused}_c${cfg}_$i -o p -- \
      python3 bench/profile_target.py ${PMC_TARGET:-fused} --reps 3 > gpurun_out/pmc/${PMC_TARGET:-fused}_c${cfg}_$i.log 2>&1
    rc=$?; echo "cfg $cfg set$i exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
