#!/bin/bash
# round 5: counter table of the heat kernels on the pitched layout (4,1) next to dense
set -o pipefail
mkdir -p gpurun_out
PMC_OUT=gpurun_out/pmc_r5p PMC_TARGETS="copy fused fused2" PMC_ARGS="--pitch 4,1" bash scripts/pmc_r5.sh > gpurun_out/pmc_r5p.log 2>&1
rc=$?
echo "exit=$rc"; tail -5 gpurun_out/pmc_r5p.log
exit $rc
