#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -m gpu tests/test_distributed_gpu.py > gpurun_out/r5/pytest_dist_bcomm.log 2>&1
rc=$?; tail -n 8 gpurun_out/r5/pytest_dist_bcomm.log; exit $rc
