#!/bin/bash
# round 5: phase-overlap variant of the fused step re-checked on the pitched layout
set -o pipefail
mkdir -p gpurun_out/r5
L=bench/ab_libs
: > gpurun_out/r5/var_pitched_ab.log
for v in fd4v19 fd4v23 fd4v7; do
  timeout -k 10 200 python -u bench/ab_step.py $L/base.so $L/$v.so --orders 4 --pitch 4,1 > gpurun_out/r5/ab_$v.log 2>&1 || { cat gpurun_out/r5/ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r5/ab_$v.log)" >> gpurun_out/r5/var_pitched_ab.log
done
for v in fd2v7 fd2v19; do
  timeout -k 10 200 python -u bench/ab_step.py $L/base.so $L/$v.so --orders 2 --pitch 4,1 > gpurun_out/r5/ab_$v.log 2>&1 || { cat gpurun_out/r5/ab_$v.log; exit 1; }
  echo "$v $(tail -1 gpurun_out/r5/ab_$v.log)" >> gpurun_out/r5/var_pitched_ab.log
done
cat gpurun_out/r5/var_pitched_ab.log
