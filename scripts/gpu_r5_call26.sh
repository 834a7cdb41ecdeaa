#!/bin/bash
# round 5: stage coefficients in VGPRs (no SGPR spills in the march) — in-process A/B
set -o pipefail
mkdir -p gpurun_out/r5
L=bench/ab_libs
: > gpurun_out/r5/vcoef_ab.log
for v in vc1 vc4; do
  timeout -k 10 200 python -u bench/ab_step.py $L/base.so $L/$v.so --pitch 4,1 --rounds 10 > gpurun_out/r5/ab_$v.log 2>&1 || { cat gpurun_out/r5/ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r5/ab_$v.log)" >> gpurun_out/r5/vcoef_ab.log
done
timeout -k 10 200 python -u bench/ab_step.py $L/vc1.so $L/base.so --pitch 4,1 --rounds 10 > gpurun_out/r5/ab_vc1_rev.log 2>&1 && echo "vc1-rev $(tail -1 gpurun_out/r5/ab_vc1_rev.log)" >> gpurun_out/r5/vcoef_ab.log
cat gpurun_out/r5/vcoef_ab.log
