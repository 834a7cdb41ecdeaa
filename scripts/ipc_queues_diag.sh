#!/bin/bash
# The Python ipc tests under different hardware-queue counts per rank (ranks share the one
# GPU).  Device waits time out after ADVDIFF_IPC_TIMEOUT_S, so a deadlock ends as a failed
# test within the step's limit.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/diag
export ADVDIFF_IPC_TIMEOUT_S=8
for q in 4 2 1; do
  ADVDIFF_TEST_HW_QUEUES=$q timeout -k 10 170 python -u -m pytest -x -v --timeout 160 --timeout-method thread \
    tests/test_ipc_gpu.py -k "slab_bitwise and diff3]" > gpurun_out/diag/pytest_q$q.log 2>&1
  rc=$?
  echo "queues=$q rc=$rc: $(grep -E 'passed|failed' gpurun_out/diag/pytest_q$q.log | tail -1)"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ]; then exit 1; fi
done
