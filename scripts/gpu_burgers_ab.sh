#!/bin/bash
# A/B of 3-D WENO5 stage kernel versions on the GPU box:
#   B3_AB="6 9" bash scripts/gpu_burgers_ab.sh
# Burgers kernel tests, interleaved stage-kernel timing (bench/burgers_variants.py), one
# PMC pass per version, and the in-solver bench with each version.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
VERS=${B3_AB:-6}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "burgers" > gpurun_out/t_burgers.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_burgers.log; exit 1; }
tail -3 gpurun_out/t_burgers.log
vlist=$(for v in $VERS; do printf "%s:8," "$v"; done); vlist=${vlist%,}
timeout -k 10 300 python -u bench/burgers_variants.py --variants "$vlist" --rounds 5 > gpurun_out/bv.log 2>&1 || { echo BVFAIL; tail -20 gpurun_out/bv.log; exit 1; }
grep -v "^{" gpurun_out/bv.log
jobs=$(for v in $VERS; do printf "burgers:ADVDIFF_B3_VER=%s " "$v"; done)
PMC_SETS_OVERRIDE='"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES" "SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"' PMC_JOBS="$jobs" bash scripts/pmc_run.sh || exit 1
python3 bench/summarize_pmc.py gpurun_out/pmc > gpurun_out/pmc_summary.md 2>&1 || true
for v in $VERS; do
  ADVDIFF_B3_VER=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-fd2 > gpurun_out/bench_v$v.log 2>&1 || { echo BENCHFAIL; tail -5 gpurun_out/bench_v$v.log; exit 1; }
  echo "v$v"; python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_v$v.log').read().strip().split('\n')[-1]); print(d['value'], d['burgers3d'])"
done
