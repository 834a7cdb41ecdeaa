#!/bin/bash
# ipc: solver rebuilt after free (regression) with and without the reset, then the whole
# ipc file and the N > 1 bench rehearsal.  Own time limit per GPU step.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export ADVDIFF_IPC_TIMEOUT_S=30
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_ipc_gpu.py > gpurun_out/pytest_ipc_rebuild.log 2>&1 || { echo "IPC TESTS FAILED"; tail -60 gpurun_out/pytest_ipc_rebuild.log; exit 1; }
tail -3 gpurun_out/pytest_ipc_rebuild.log
NS="${NS:-2 4 8}" bash scripts/bench_rehearsal_ipc.sh
