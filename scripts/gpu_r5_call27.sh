#!/bin/bash
# round 5: stage-1 coefficients in VGPRs (spill-free fused step) — tests, bench, counters,
# and the FD2 8 x 3 tile (spill-free now) re-checked
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_fused_step_gpu.py tests/test_pitch_gpu.py > gpurun_out/r5/vcoef_tests.log 2>&1 && \
ADVDIFF_STEP_BANDS_LOG=1 ADVDIFF_STEP2_LOG=1 timeout -k 10 300 python -u bench.py > gpurun_out/r5/bench6.log 2>&1 && \
timeout -k 10 300 python -u bench/step_tile_ab.py --alt 1 --pitch 4,1 --sizes 384,512,768 > gpurun_out/r5/step_tile_ab_vcoef.log 2>&1 && \
PMC_OUT=gpurun_out/pmc_r5v PMC_TARGETS="fused fused2 step2x" PMC_ARGS="--pitch 4,1" bash scripts/pmc_r5.sh > gpurun_out/pmc_r5v.log 2>&1
rc=$?
echo "exit=$rc"; tail -2 gpurun_out/r5/vcoef_tests.log; grep advdiff gpurun_out/r5/bench6.log
grep -o '"value": [0-9.]*, "unit": "MLUPS", "n_gpus"\|"fd2_7pt": {"value": [0-9.]*\|"burgers3d": {"value": [0-9.]*\|"sustained": {"steps": 200, "value": [0-9.]*' gpurun_out/r5/bench6.log
cat gpurun_out/r5/step_tile_ab_vcoef.log
exit $rc
