#!/bin/bash
# round 5: banded z schedule of the fused step — tests, then the A/B
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_fused_step_gpu.py > gpurun_out/r5/banded_tests.log 2>&1 && \
ADVDIFF_STEP_BANDS_LOG=1 timeout -k 10 500 python -u bench/banded_ab.py > gpurun_out/r5/banded_ab.log 2>&1
rc=$?
echo "exit=$rc"; tail -3 gpurun_out/r5/banded_tests.log; cat gpurun_out/r5/banded_ab.log
exit $rc
