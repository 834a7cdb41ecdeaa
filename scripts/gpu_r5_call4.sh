#!/bin/bash
# ipc tests with the comm-stream boundary as the ipc default; chunk sweeps (FD2 two-step,
# WENO5 stage)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5/ab
export PYTHONUNBUFFERED=1
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  -m gpu tests/test_ipc_gpu.py tests/test_distributed_gpu.py > gpurun_out/r5/pytest_ipc_bcomm.log 2>&1
rc=$?; tail -n 15 gpurun_out/r5/pytest_ipc_bcomm.log; [ $rc -eq 0 ] || exit $rc
echo "== step2 chunks"
timeout -k 10 240 python bench/step2_chunks.py --n 512 > gpurun_out/r5/ab/step2_chunks.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5/ab/step2_chunks.log | head -12
echo "== b3 chunks"
timeout -k 10 300 python bench/b3_chunk_sweep.py --sizes 256,512 --chunks 0,32,42,50,63,64,85,102 --rounds 5 \
  > gpurun_out/r5/ab/b3_chunk_sweep2.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5/ab/b3_chunk_sweep2.log | head -40
