#!/bin/bash
# round 5: pitch candidates for the default, two processes with opposite orders
set -o pipefail
mkdir -p gpurun_out/r5
P="0,0 4,1 8,1 8,3 4,3 2,3 16,3 2,1 24,1 8,2"
R="8,2 24,1 2,1 16,3 2,3 4,3 8,3 8,1 4,1 0,0"
timeout -k 10 400 python -u bench/pitch_ab.py --n 512 --rounds 5 --pads $P > gpurun_out/r5/pitch_cand_a.log 2>&1 && \
timeout -k 10 400 python -u bench/pitch_ab.py --n 512 --rounds 5 --pads $R > gpurun_out/r5/pitch_cand_b.log 2>&1
rc=$?
echo "exit=$rc"; cat gpurun_out/r5/pitch_cand_a.log gpurun_out/r5/pitch_cand_b.log | cut -c1-200
exit $rc
