#!/bin/bash
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_step_gpu.py tests/test_kernels_gpu.py -k "fused or burgers3d" > gpurun_out/pytest_ab.log 2>&1 || { echo "TESTS FAILED"; tail -30 gpurun_out/pytest_ab.log; exit 1; }
tail -1 gpurun_out/pytest_ab.log
timeout -k 10 300 python -u bench/burgers_ab.py > gpurun_out/burgers_ab.log 2>&1 || { echo "BURGERS AB FAILED"; tail -20 gpurun_out/burgers_ab.log; exit 1; }
grep '^{' gpurun_out/burgers_ab.log
timeout -k 10 300 python -u bench/step_ab.py > gpurun_out/step_ab.log 2>&1 || { echo "STEP AB FAILED"; tail -20 gpurun_out/step_ab.log; exit 1; }
grep '^{' gpurun_out/step_ab.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo "BENCH FAILED"; tail -20 gpurun_out/bench.log; exit 1; }
grep '^{' gpurun_out/bench.log
