#!/bin/bash
# Round-3 stall breakdown of the hot kernels (bench/profile_target.py targets), one
# counter group per rocprofv3 run (--pmc with kernel trace only), plus the counter list.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
out=${PMC_OUT:-gpurun_out/pmc_r3}
mkdir -p $out
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || echo "counter list rc=$?"
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
      "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES"
      "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE GRBM_COUNT"
      "FETCH_SIZE"
      "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum")
for tgt in ${PMC_TARGETS:-fused fused2 burgers}; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $out/${tgt}_$i -o p -- \
      python3 bench/profile_target.py $tgt --reps 3 > $out/${tgt}_$i.log 2>&1
    rc=$?; echo "$tgt set$i exit $rc"
    if [ $rc -ne 0 ]; then tail -5 $out/${tgt}_$i.log; fi
  done
done
