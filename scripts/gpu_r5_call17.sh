#!/bin/bash
# round 5: solver-level pitch candidates, two processes with opposite orders
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u bench/pitch_solver_ab.py --cases fd4 fd2 --rounds 5 --pitches 0,0 8,1 4,1 2,1 2,3 4,3 > gpurun_out/r5/pitch_solver_c_a.log 2>&1 && \
timeout -k 10 400 python -u bench/pitch_solver_ab.py --cases fd4 fd2 --rounds 5 --pitches 4,3 2,3 2,1 4,1 8,1 0,0 > gpurun_out/r5/pitch_solver_c_b.log 2>&1
rc=$?
echo "exit=$rc"
exit $rc
