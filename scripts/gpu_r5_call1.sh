#!/bin/bash
# determinism diagnosis (bounded; rc 0/1 = ran) then the full GPU suite
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u bench/burgers_determinism.py > gpurun_out/r5/burgers_determinism.log 2>&1
rc=$?
echo "determinism rc=$rc"; tail -n 4 gpurun_out/r5/burgers_determinism.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
SUITE_LIMIT=${SUITE_LIMIT:-840} bash scripts/gpu_r5_suite.sh
