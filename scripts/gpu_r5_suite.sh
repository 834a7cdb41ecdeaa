#!/bin/bash
# Full GPU test suite at HEAD, one bounded pytest process, per-test durations kept.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5
timeout -k 10 ${SUITE_LIMIT:-1080} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread --durations=60 ${SUITE_ARGS:-} \
  > gpurun_out/r5/pytest_gpu.log 2>&1
rc=$?
tail -n 80 gpurun_out/r5/pytest_gpu.log
exit $rc
