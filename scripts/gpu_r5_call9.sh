#!/bin/bash
# round 5: device-dt over ipc (both schedules), fp32 heat tile A/B, 3-D size sweep
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_adaptive_dt.py -m gpu > gpurun_out/r5/adaptive_ipc.log 2>&1 && \
timeout -k 10 240 python -u bench/step_fp32_ab.py > gpurun_out/r5/step_fp32_ab.log 2>&1 && \
timeout -k 10 400 python -u bench/sizes3d.py > gpurun_out/r5/sizes3d.log 2>&1
rc=$?
echo "exit=$rc"; tail -3 gpurun_out/r5/adaptive_ipc.log; cat gpurun_out/r5/step_fp32_ab.log gpurun_out/r5/sizes3d.log 2>/dev/null
exit $rc
