#!/bin/bash
# round 5: u/v relative placement (one allocation, chosen distance) vs pitch
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 400 python -u bench/alias_ab.py > gpurun_out/r5/alias_ab.log 2>&1
rc=$?
echo "exit=$rc"; cut -c1-200 gpurun_out/r5/alias_ab.log
exit $rc
