#!/bin/bash
# Native engine hipGraph stepping (single rank and ipc multi-rank) + the fused-step PMC
# stall counters (current defaults and the plain VAR 0 kernel).  Own time limit per step.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread \
  tests/test_native_apps_gpu.py > gpurun_out/pytest_native_graph.log 2>&1 || { echo "TESTS FAILED"; tail -60 gpurun_out/pytest_native_graph.log; exit 1; }
tail -3 gpurun_out/pytest_native_graph.log
if [ "${PMC:-1}" = "1" ]; then
  PMC_OUT=gpurun_out/pmc_r3b PMC_TARGETS="fused fused2" bash scripts/pmc_r3.sh && \
  ADVDIFF_STEP_VAR=0 PMC_OUT=gpurun_out/pmc_r3b_var0 PMC_TARGETS="fused fused2" bash scripts/pmc_r3.sh
fi
