#!/bin/bash
# FD2 tile A/B (8x3, two workgroups per CU, vs 12x3), then the N = 2 / 4 rehearsal
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5/ab
timeout -k 10 300 python bench/step_tile_ab.py > gpurun_out/r5/ab/step_fd2_tile_ab.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5/ab/step_fd2_tile_ab.log
bash scripts/gpu_r5_rehearsal.sh
