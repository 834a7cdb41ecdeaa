#!/bin/bash
# round 5: default pitch 4 fp64 / 16 fp32 elements + 1 row — tests and bench
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_pitch_gpu.py tests/test_native_apps_gpu.py -k "pitch or field_memory or matches_python" > gpurun_out/r5/pitch_tests3.log 2>&1 && \
timeout -k 10 300 python -u bench.py > gpurun_out/r5/bench4.log 2>&1
rc=$?
echo "exit=$rc"; tail -4 gpurun_out/r5/pitch_tests3.log; tail -1 gpurun_out/r5/bench4.log | cut -c1-1500
exit $rc
