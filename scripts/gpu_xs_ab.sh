#!/bin/bash
# Fused step: x neighbours of stages 2/3 from LDS (XS = 0, VAR + 64) vs DPP — bitwise tests,
# then the interleaved A/B for FD4 and FD2.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_fused_step_gpu.py > gpurun_out/pytest_xs.log 2>&1 || { echo "STEP TESTS FAILED"; tail -40 gpurun_out/pytest_xs.log; exit 1; }
tail -2 gpurun_out/pytest_xs.log
timeout -k 10 500 python -u bench/step_ab.py --rounds 7 --reps 10 --vars ${VARS:-3,67,83,80} --orders ${ORDERS:-4,2} > gpurun_out/step_ab_xs.log 2>&1 || { echo "A/B FAILED"; tail -20 gpurun_out/step_ab_xs.log; exit 1; }
tail -2 gpurun_out/step_ab_xs.log
