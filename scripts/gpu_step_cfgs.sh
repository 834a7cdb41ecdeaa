#!/bin/bash
# Fused-step tile-config A/B with edge tiles (grid schedule), interleaved rounds.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u bench/step_variants.py --cfgs ${CFGS:-0,29,31,32,33} --edges 1 --schedules grid --rounds 5 --reps 10 > gpurun_out/step_cfgs.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/step_cfgs.log; exit 1; }
grep -v "^{" gpurun_out/step_cfgs.log
