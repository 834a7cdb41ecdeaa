#!/bin/bash
# Round 5: kernel-trace stats of the hot kernels (one run), then per-kernel counter passes
# (one group per rocprofv3 --pmc run, kernel trace only, each under its own limit):
# the stall split of round 3 (set 1), clock (set 2) and the fabric bytes of round 4
# (set 3) for copy (calibration), fused FD4, fused FD2, the two-step FD2 launch and the
# WENO5-Z viscous stage.  PMC_OUT / PMC_TARGETS / PMC_ARGS (e.g. "--pitch 4,1": the
# solver's pitched layout) select the output, the kernels and the field layout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out=${PMC_OUT:-gpurun_out/pmc_r5}
mkdir -p $out
for tgt in ${PMC_TARGETS:-copy fused fused2 step2x burgers}; do
  timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $out/${tgt}_trace -o p -- \
    python3 bench/profile_target.py $tgt --reps 8 ${PMC_ARGS:-} > $out/${tgt}_trace.log 2>&1
  rc=$?; echo "$tgt trace exit $rc"; [ $rc -eq 0 ] || { tail -5 $out/${tgt}_trace.log; exit $rc; }
done
SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES"
      "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
      "TCC_EA0_RDREQ_sum WRITE_SIZE")
for tgt in ${PMC_TARGETS:-copy fused fused2 step2x burgers}; do
  i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $out/${tgt}_$i -o p -- \
      python3 bench/profile_target.py $tgt --reps 5 ${PMC_ARGS:-} > $out/${tgt}_$i.log 2>&1
    rc=$?; echo "$tgt set$i exit $rc"
    if [ $rc -ne 0 ]; then tail -5 $out/${tgt}_$i.log; exit $rc; fi
  done
done
python3 bench/summarize_pmc.py $out > $out/summary.md
