#!/bin/bash
# round 5: pitched fields by default (3-D, > 128 MiB per rank) — Python + native tests,
# the solver A/B against pitch 0,0, and the bench
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_pitch_gpu.py tests/test_native_apps_gpu.py -k "pitch or field_memory or matches_python" > gpurun_out/r5/pitch_tests2.log 2>&1 && \
timeout -k 10 400 python -u bench/pitch_solver_ab.py --pitches 0,0 8,1 --cases fd4 fd2 --rounds 5 > gpurun_out/r5/pitch_solver_ab2.log 2>&1 && \
timeout -k 10 400 python -u bench/pitch_ab.py --n 512 --dtype fp32 --pads 0,0 16,0 16,1 8,1 > gpurun_out/r5/pitch_ab_fp32.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r5/bench3.log 2>&1
rc=$?
echo "exit=$rc"; tail -4 gpurun_out/r5/pitch_tests2.log; cat gpurun_out/r5/pitch_solver_ab2.log gpurun_out/r5/pitch_ab_fp32.log 2>/dev/null; tail -2 gpurun_out/r5/bench3.log | cut -c1-1500
exit $rc
