#!/bin/bash
# PMC counter passes (kernel-trace only, no sys/runtime traces) for the hot kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
[ -f "${PMC_SETS_FILE:-scripts/pmc_sets.sh}" ] && source "${PMC_SETS_FILE:-scripts/pmc_sets.sh}"
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
for tgt in ${PMC_TARGETS:-fused burgers}; do
  i=0
  for set in "${PMC_SETS[@]:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES}"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/${tgt}_$i -o p -- \
      python3 bench/profile_target.py $tgt --reps 3 > gpurun_out/pmc/${tgt}_$i.log 2>&1
    rc=$?; echo "$tgt set$i exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
