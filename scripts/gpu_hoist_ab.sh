#!/bin/bash
# FD2 HOIST variants: bitwise tests, then the interleaved step A/B (FD2 only matters).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_fused_step_gpu.py > gpurun_out/pytest_hoist.log 2>&1 || { echo "STEP TESTS FAILED"; tail -40 gpurun_out/pytest_hoist.log; exit 1; }
tail -2 gpurun_out/pytest_hoist.log
timeout -k 10 400 python -u bench/step_ab.py --rounds 7 --reps 10 --vars 23,55,51,7 --orders 2 > gpurun_out/step_ab_hoist.log 2>&1 || { echo "A/B FAILED"; tail -20 gpurun_out/step_ab_hoist.log; exit 1; }
tail -2 gpurun_out/step_ab_hoist.log
