#!/bin/bash
# round 5: fp32 heat tile default (FD4 16 x 4) — tests and the size sweep of the A/B;
# pitched-allocation A/B of the fused heat step
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_fused_step_gpu.py > gpurun_out/r5/fused_step_fp32.log 2>&1 && \
timeout -k 10 400 python -u bench/step_fp32_ab.py --n 256 384 512 640 768 1024 > gpurun_out/r5/step_fp32_ab.log 2>&1 && \
timeout -k 10 300 python -u bench/pitch_ab.py --n 512 384 > gpurun_out/r5/pitch_ab.log 2>&1
rc=$?
echo "exit=$rc"; tail -3 gpurun_out/r5/fused_step_fp32.log; cat gpurun_out/r5/step_fp32_ab.log gpurun_out/r5/pitch_ab.log 2>/dev/null
exit $rc
