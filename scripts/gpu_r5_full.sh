#!/bin/bash
# Full GPU suite at HEAD (one bounded pytest process), then smoke and the default bench.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5
export PYTHONUNBUFFERED=1
timeout -k 10 ${SUITE_LIMIT:-900} python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread --durations=25 > gpurun_out/r5/pytest_gpu_full.log 2>&1
rc=$?; tail -n 35 gpurun_out/r5/pytest_gpu_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python __graft_entry__.py smoke > gpurun_out/r5/smoke.log 2>&1 || exit $?
tail -n 4 gpurun_out/r5/smoke.log
ADVDIFF_STEP2_LOG=1 timeout -k 10 400 python bench.py > gpurun_out/r5/bench_full.log 2>&1
rc=$?; tail -c 2500 gpurun_out/r5/bench_full.log; [ $rc -eq 0 ] || exit $rc
[ -n "$NO_PMC" ] || bash scripts/pmc_r5.sh
