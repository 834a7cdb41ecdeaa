#!/bin/bash
# FD2 12x4 (48-row) tile A/B and its bitwise tests
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5/ab
timeout -k 10 300 python bench/step_tile_ab.py --alt 2 --sizes 384,512,640,768,1024 \
  > gpurun_out/r5/ab/step_tile_ab_12x4.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5/ab/step_tile_ab_12x4.log
ADVDIFF_STEP_FD2_TILE=2 timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -m gpu tests/test_fused_step_gpu.py > gpurun_out/r5/pytest_fused_12x4.log 2>&1
rc=$?; tail -n 5 gpurun_out/r5/pytest_fused_12x4.log; exit $rc
