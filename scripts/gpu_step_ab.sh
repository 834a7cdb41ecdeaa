#!/bin/bash
# Fused-step phase-overlap variants: bitwise tests, interleaved kernel A/B, bench per variant.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fused_step_gpu.py > gpurun_out/pytest_step.log 2>&1 || { echo "STEP TESTS FAILED"; tail -30 gpurun_out/pytest_step.log; exit 1; }
tail -1 gpurun_out/pytest_step.log
timeout -k 10 400 python -u bench/step_ab.py --rounds 7 --reps 10 > gpurun_out/step_ab.log 2>&1 || { echo "STEP AB FAILED"; tail -20 gpurun_out/step_ab.log; exit 1; }
cat gpurun_out/step_ab.log | grep '^{'
for v in ${BENCH_VARS:-0 -1}; do
  ADVDIFF_STEP_VAR=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_var$v.log 2>&1 || { echo "BENCH var $v FAILED"; tail -20 gpurun_out/bench_var$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/bench_var$v.log') if l.startswith('{')][-1]); print('var $v', d['value'], d['ms_per_step'], 'sustained', d['sustained']['value'], 'fd2', d['fd2_7pt']['value'])"
done
