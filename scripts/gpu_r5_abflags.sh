#!/bin/bash
# in-process A/Bs of compiler-scheduler variants of the kernel library (bench/ab_libs)
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5/ab
for v in ${VARIANTS:-maxilp memclause}; do
  echo "== step base vs $v"
  timeout -k 10 200 python bench/ab_step.py bench/ab_libs/base.so bench/ab_libs/$v.so --rounds 8 \
    > gpurun_out/r5/ab/abflags_step_$v.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r5/ab/abflags_step_$v.log | tail -3
  echo "== burgers base vs $v"
  timeout -k 10 200 python bench/ab_burgers.py bench/ab_libs/base.so bench/ab_libs/$v.so --rounds 6 \
    > gpurun_out/r5/ab/abflags_burgers_$v.log 2>&1 || exit $?
  grep -v amdgpu.ids gpurun_out/r5/ab/abflags_burgers_$v.log | tail -3
done
