#!/bin/bash
# round 5: stage coefficients in VGPRs (no SGPR spills in the march) — in-process A/B
set -o pipefail
mkdir -p gpurun_out/r5
L=bench/ab_libs
: > gpurun_out/r5/vcoef_ab2.log
for v in vc3 vc5; do
  timeout -k 10 200 python -u bench/ab_step.py $L/base.so $L/$v.so --pitch 4,1 --rounds 10 > gpurun_out/r5/ab_$v.log 2>&1 || { cat gpurun_out/r5/ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r5/ab_$v.log)" >> gpurun_out/r5/vcoef_ab2.log
done

cat gpurun_out/r5/vcoef_ab2.log
