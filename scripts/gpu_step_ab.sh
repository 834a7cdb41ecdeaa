#!/bin/bash
# Fused-step A/B on one GPU: bitwise tests of the fused step, edge tiles on/off timing,
# then the bench (scripts/gpu_step_ab.sh; results under gpurun_out/).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_step_gpu.py > gpurun_out/t_step.log 2>&1 || { echo TESTFAIL; tail -30 gpurun_out/t_step.log; exit 1; }
tail -2 gpurun_out/t_step.log
timeout -k 10 300 python -u bench/step_variants.py --cfgs 0 --edges 1,0 --schedules grid,persist --rounds 5 --reps 10 > gpurun_out/step_ab.log 2>&1 || { echo ABFAIL; tail -20 gpurun_out/step_ab.log; exit 1; }
grep -v "^{" gpurun_out/step_ab.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo BENCHFAIL; tail -5 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log | cut -c1-300
