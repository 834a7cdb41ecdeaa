#!/bin/bash
# Fused step: adjacent-row (PAIR) variants — bitwise tests, then the interleaved A/B; then
# the ipc regression + bench rehearsal.  Own time limit per GPU step.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_fused_step_gpu.py > gpurun_out/pytest_pair.log 2>&1 || { echo "STEP TESTS FAILED"; tail -40 gpurun_out/pytest_pair.log; exit 1; }
tail -2 gpurun_out/pytest_pair.log
timeout -k 10 400 python -u bench/step_ab.py --rounds 7 --reps 10 --vars ${VARS:-3,23,7,0} > gpurun_out/step_ab_pair.log 2>&1 || { echo "A/B FAILED"; tail -20 gpurun_out/step_ab_pair.log; exit 1; }
tail -3 gpurun_out/step_ab_pair.log
if [ "${REBUILD:-1}" = "1" ]; then bash scripts/gpu_ipc_rebuild.sh; fi
