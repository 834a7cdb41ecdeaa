#!/bin/bash
# Roofline evidence: kernel-trace timings + PMC passes (kernel-trace only, one counter
# group per run) of bench/roofline_targets.py; summarised by bench/roofline_table.py into
# profiles/roofline.md.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/roofline
mkdir -p $out
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $out/trace -o t -- \
  python3 bench/roofline_targets.py --reps 5 > $out/trace.log 2>&1 || exit $?
i=0
for set in "FETCH_SIZE" "WRITE_SIZE TCC_EA0_RDREQ_sum" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "TCC_EA0_RDREQ_32B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $out/pmc_$i -o p -- \
    python3 bench/roofline_targets.py --reps 3 > $out/pmc_$i.log 2>&1
  rc=$?; echo "set$i exit $rc"; [ $rc -eq 0 ] || exit $rc
done
