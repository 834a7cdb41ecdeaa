#!/bin/bash
# round 5: counter table of the heat kernels on the pitched layout (4,1) next to dense
set -o pipefail
mkdir -p gpurun_out/r5
PMC_OUT=gpurun_out/pmc_r5p PMC_TARGETS="copy fused fused2" PMC_ARGS="--pitch 4,1" bash scripts/pmc_r5.sh > gpurun_out/pmc_r5p.log 2>&1
rc=$?
[ $rc -eq 0 ] && { timeout -k 10 300 python -u bench/pitch_ab.py --dims 2 --n 8192 16384 --rounds 4 --pads 0,0 4,0 8,0 16,0 32,0 > gpurun_out/r5/pitch_ab_2d.log 2>&1; rc=$?; }
echo "exit=$rc"; tail -5 gpurun_out/pmc_r5p.log; cat gpurun_out/r5/pitch_ab_2d.log
exit $rc
