#!/bin/bash
# XCD-balanced uneven z chunks of the fused step (ADVDIFF_STEP_SPLIT=1) vs uniform chunks
# (=0): bitwise step tests with the split on, then alternating kernel timings (bench/
# step_ab.py, FD4 and FD2 512^3) and 20-step bench windows.  Own time limit per step.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
: > gpurun_out/split_ab.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_fused_step_gpu.py > gpurun_out/pytest_split.log 2>&1 || { echo "STEP TESTS FAILED"; tail -30 gpurun_out/pytest_split.log; exit 1; }
tail -1 gpurun_out/pytest_split.log
for r in 1 2 3; do
  for v in 0 1; do
    ADVDIFF_STEP_SPLIT=$v timeout -k 10 200 python -u bench/step_ab.py --vars -1 --rounds 3 --reps 10 > gpurun_out/split_k$v.log 2>&1 || { echo "STEP AB $v FAILED"; tail -20 gpurun_out/split_k$v.log; exit 1; }
    echo "kernel split=$v $(grep '^{' gpurun_out/split_k$v.log | tr '\n' ' ')" >> gpurun_out/split_ab.log
    ADVDIFF_STEP_SPLIT=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-burgers --sustained-steps 100 > gpurun_out/split_b$v.log 2>&1 || { echo "BENCH $v FAILED"; tail -20 gpurun_out/split_b$v.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/split_b$v.log') if l.startswith('{')][-1]); print('bench split=$v', d['value'], d['ms_per_step'], 'sustained', d['sustained']['value'], 'fd2', d['fd2_7pt']['value'])" >> gpurun_out/split_ab.log
  done
done
cat gpurun_out/split_ab.log
