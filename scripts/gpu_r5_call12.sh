#!/bin/bash
# round 5: pitched device fields — bitwise tests, then the solver-level pitch A/B
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_pitch_gpu.py > gpurun_out/r5/pitch_tests.log 2>&1 && \
timeout -k 10 500 python -u bench/pitch_solver_ab.py > gpurun_out/r5/pitch_solver_ab.log 2>&1
rc=$?
echo "exit=$rc"; tail -5 gpurun_out/r5/pitch_tests.log; cat gpurun_out/r5/pitch_solver_ab.log 2>/dev/null
exit $rc
