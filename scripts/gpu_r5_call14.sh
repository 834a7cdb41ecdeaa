#!/bin/bash
# round 5: finer pitch sweep of the FD4 fused step at 512^3 (the headline)
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u bench/pitch_ab.py --n 512 --orders 4 --rounds 5 --pads 0,0 4,1 8,1 2,1 6,1 12,1 4,3 8,3 8,5 4,7 8,7 24,1 8,9 8,17 > gpurun_out/r5/pitch_sweep_fd4.log 2>&1 && \
timeout -k 10 400 python -u bench/pitch_ab.py --n 512 --orders 2 --rounds 5 --pads 0,0 4,1 8,1 2,1 6,1 12,1 4,3 8,3 8,5 4,7 8,7 24,1 8,9 8,17 > gpurun_out/r5/pitch_sweep_fd2.log 2>&1
rc=$?
echo "exit=$rc"; cat gpurun_out/r5/pitch_sweep_fd4.log gpurun_out/r5/pitch_sweep_fd2.log | cut -c1-220
exit $rc
