#!/bin/bash
# PMC passes (kernel-trace only, one counter group per run) of bench/profile_target.py
# targets under environment variants:
#   PMC_JOBS="burgers:ADVDIFF_B3_VER=1 burgers:ADVDIFF_B3_VER=3 fused:ADVDIFF_STEP_CFG=0" \
#     bash scripts/pmc_run.sh
# Output: gpurun_out/pmc/<tag>_<set>/p_counter_collection.csv, summarised by
# bench/summarize_pmc.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
      "FETCH_SIZE"
      "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum")
[ -n "$PMC_SETS_OVERRIDE" ] && eval "SETS=($PMC_SETS_OVERRIDE)"
for job in ${PMC_JOBS:-burgers:ADVDIFF_B3_VER=2}; do
  tgt=${job%%:*}; envs=${job#*:}; envs=${envs//,/ }
  tag="${tgt}_$(echo "$envs" | tr -c 'A-Za-z0-9\n' '_' | sed 's/ADVDIFF_//g')"
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    (export $envs; timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv \
      -d gpurun_out/pmc/${tag}_$i -o p -- \
      python3 bench/profile_target.py $tgt --reps 3 > gpurun_out/pmc/${tag}_$i.log 2>&1)
    rc=$?; echo "$tag set$i exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
