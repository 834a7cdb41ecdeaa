#!/bin/bash
# the GPU test files the first round-5 suite run did not reach, then the A/Bs
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=30 -m gpu tests/test_kernels_gpu.py tests/test_lu_exchange.py tests/test_native_apps_gpu.py \
  tests/test_rccl_multirank.py tests/test_weno7_lsrk_gpu.py "tests/test_ipc_gpu.py::test_native_boundary_on_comm_bitwise" \
  > gpurun_out/r5/pytest_gpu_part2.log 2>&1
rc=$?
tail -n 40 gpurun_out/r5/pytest_gpu_part2.log
[ $rc -eq 0 ] || exit $rc
AB_STEPS="step2 fp32weno tile" bash scripts/gpu_r5_ab.sh
