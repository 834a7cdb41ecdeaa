#!/bin/bash
# Direct (one-phase, diagonal neighbours) vs phased corner exchange: IPC + native + RCCL
# multi-rank GPU tests.  Every GPU step has its own time limit.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export ADVDIFF_IPC_TIMEOUT_S=${ADVDIFF_IPC_TIMEOUT_S:-30}
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_ipc_gpu.py tests/test_distributed_gpu.py tests/test_native_apps_gpu.py \
  > gpurun_out/pytest_corners.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/pytest_corners.log; exit 1; }
tail -3 gpurun_out/pytest_corners.log
