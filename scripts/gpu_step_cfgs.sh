#!/bin/bash
# Fused-step tile/x-source config A/B (grid schedule, edge tiles), interleaved rounds,
# after the fused-step bitwise tests.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_step_gpu.py > gpurun_out/t_step.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_step.log; exit 1; }
tail -1 gpurun_out/t_step.log
timeout -k 10 400 python -u bench/step_variants.py --cfgs ${CFGS:-29,34,35,38,30,36,37,39} --edges 1 --schedules grid --rounds 5 --reps 10 > gpurun_out/step_cfgs.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/step_cfgs.log; exit 1; }
grep -v "^{" gpurun_out/step_cfgs.log
