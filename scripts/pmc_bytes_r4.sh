#!/bin/bash
# Round 4: ONE harness (bench/profile_target.py: the bench's 512^3 fp64 launch of the fused
# step, single-rank full range) and ONE launch shape for every byte counter of the fused
# FD4 / FD2 step, with the copy kernel as the calibration (exactly n^3 x 8 B each way).
# One rocprofv3 --pmc run per counter group (kernel trace only), each under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=${PMC_OUT:-gpurun_out/pmc_bytes_r4}
mkdir -p $out
timeout -s KILL 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || echo "counter list rc=$?"
SETS=("TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
      "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE"
      "FETCH_SIZE GRBM_GUI_ACTIVE"
      "WRITE_SIZE TCC_EA0_RDREQ_sum")
if grep -q "TCC_EA0_RDREQ_DRAM" $out/counters_list.txt; then
  SETS+=("TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum")
fi
for tgt in copy fused fused2; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $out/${tgt}_$i -o p -- \
      python3 bench/profile_target.py $tgt --reps 5 > $out/${tgt}_$i.log 2>&1
    rc=$?; echo "$tgt set$i exit $rc"
    if [ $rc -ne 0 ]; then tail -5 $out/${tgt}_$i.log; exit $rc; fi
  done
done
python3 bench/summarize_pmc.py $out > $out/summary.md
