#!/bin/bash
# Kernel sweep: each configuration (ADVDIFF_* settings, '+'-joined) in its own process
# (knobs are read once per process), e.g. KB_CONFIGS="ADVDIFF_B3_VER=9 ADVDIFF_B3_VER=3".
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -x -q > gpurun_out/kt.log 2>&1; rc=$?; tail -2 gpurun_out/kt.log
case $rc in 0|1) ;; *) exit $rc;; esac
for cfg in ${KB_CONFIGS:-"ADVDIFF_B3_VER=9"}; do
  echo "== $cfg" | tee -a gpurun_out/kbench.log
  env ${cfg//+/ } timeout -k 10 120 python bench/kernels.py ${KB_ARGS:-} >> gpurun_out/kbench.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { echo "exit $rc"; exit $rc; }
done
cat gpurun_out/kbench.log
