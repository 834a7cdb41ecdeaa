#!/bin/bash
# round 5: pitched-allocation sweep of the fused heat step (row pad px elements, plane pad py rows)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u bench/pitch_ab.py --n 512 --rounds 3 --pads 0,0 1,0 4,0 8,0 16,0 24,0 32,0 40,0 0,1 1,1 4,1 8,1 16,1 32,1 8,2 16,2 8,3 > gpurun_out/r5/pitch_sweep512.log 2>&1 && \
timeout -k 10 300 python -u bench/pitch_ab.py --n 256 640 768 --rounds 3 --pads 0,0 8,0 16,0 8,1 16,1 > gpurun_out/r5/pitch_sweep_sizes.log 2>&1
rc=$?
echo "exit=$rc"; cat gpurun_out/r5/pitch_sweep512.log gpurun_out/r5/pitch_sweep_sizes.log 2>/dev/null | cut -c1-200
exit $rc
