#!/bin/bash
# Round 4 perf probes: fused-step z-chunk sweep (512^3, 1024^3, 8-GPU slab block), the
# Burgers tile-row A/B, then the one-harness byte counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench/step_chunks.py --rounds 2 > gpurun_out/step_chunks.log 2>&1 || { echo "step_chunks rc=$?"; tail -20 gpurun_out/step_chunks.log; exit 1; }
cat gpurun_out/step_chunks.log
bash scripts/pmc_bytes_r4.sh || exit 1
cat gpurun_out/pmc_bytes_r4/summary.md
