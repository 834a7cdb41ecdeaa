#!/bin/bash
# Round-3 final evidence: rocprofv3 kernel stats of the bench, and the native executables
# at the bench sizes with and without hipGraph stepping.  Own time limit per step.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
PROF_NAME=r3final BENCH_ARGS="--steps 20 --warmup 5 --sustained-steps 0" bash scripts/profile.sh || exit 1
: > gpurun_out/native_r3.log
for g in --graph --no-graph; do
  RANK=0 WORLD_SIZE=1 timeout -k 10 120 bin/diffusion3d 1 1 1 1 512 512 512 200 --ic sine $g >> gpurun_out/native_r3.log 2>&1 || exit 1
  RANK=0 WORLD_SIZE=1 timeout -k 10 120 bin/diffusion3d 1 1 1 1 512 512 512 200 --ic sine --order 2 $g >> gpurun_out/native_r3.log 2>&1 || exit 1
  RANK=0 WORLD_SIZE=1 timeout -k 10 120 bin/burgers3d 0.05 0.3 2 2 2 256 256 256 --weno z --visc 1e-5 $g >> gpurun_out/native_r3.log 2>&1 || exit 1
done
grep -E "Optimization|Computation|Time steps|MLUPS|Total|native build" gpurun_out/native_r3.log | head -60
