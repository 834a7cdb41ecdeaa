#!/bin/bash
# round 5: measured banded/uniform schedule — tests, A/B, bench with the picks logged
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_fused_step_gpu.py tests/test_pitch_gpu.py > gpurun_out/r5/sched_tests.log 2>&1 && \
timeout -k 10 500 python -u bench/banded_ab.py > gpurun_out/r5/banded_ab2.log 2>&1 && \
ADVDIFF_STEP_BANDS_LOG=1 ADVDIFF_STEP2_LOG=1 timeout -k 10 300 python -u bench.py > gpurun_out/r5/bench5.log 2>&1
rc=$?
echo "exit=$rc"; tail -3 gpurun_out/r5/sched_tests.log; cat gpurun_out/r5/banded_ab2.log; grep advdiff gpurun_out/r5/bench5.log; tail -1 gpurun_out/r5/bench5.log | cut -c1-300
grep -o '"fd2_7pt": {"value": [0-9.]*\|"burgers3d": {"value": [0-9.]*\|"sustained": {"steps": 200, "value": [0-9.]*' gpurun_out/r5/bench5.log
exit $rc
