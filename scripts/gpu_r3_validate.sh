#!/bin/bash
# Round-3 GPU validation: IPC transport + poisoned native multi-rank tests first, then the
# whole GPU suite, the driver's smoke(), then the headline bench.  Every GPU step has its own time limit.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export ADVDIFF_IPC_TIMEOUT_S=${ADVDIFF_IPC_TIMEOUT_S:-30}
if [ "${IPC:-1}" = "1" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_ipc_gpu.py > gpurun_out/pytest_ipc.log 2>&1 || { echo "IPC TESTS FAILED"; tail -60 gpurun_out/pytest_ipc.log; exit 1; }
  tail -3 gpurun_out/pytest_ipc.log
fi
if [ "${FULL:-1}" = "1" ]; then
  timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/ > gpurun_out/pytest_gpu.log 2>&1 || { echo "GPU SUITE FAILED"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
fi
if [ "${SMOKE:-1}" = "1" ]; then
  timeout -k 10 300 python -u __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 || { echo "SMOKE FAILED"; tail -30 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -30 gpurun_out/bench.log; exit 1; }
  tail -2 gpurun_out/bench.log
fi
