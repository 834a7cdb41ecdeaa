#!/bin/bash
# overlap traces, FD2 two-step crossover sizes, WENO5 z-chunk sweep, then bench.py
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out/r5/ab
export PYTHONUNBUFFERED=1
bash scripts/gpu_r5_overlap.sh || exit $?
echo "== step2 sizes"
timeout -k 10 300 python bench/step2_ab.py --sizes 384,640,768,896 --dtypes float64 --rounds 3 \
  > gpurun_out/r5/ab/step2_sizes.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5/ab/step2_sizes.log
echo "== b3 chunk sweep"
timeout -k 10 300 python bench/b3_chunk_sweep.py --sizes 256,512 --rounds 2 \
  > gpurun_out/r5/ab/b3_chunk_sweep.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/r5/ab/b3_chunk_sweep.log | head -8
echo "== bench"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r5/bench1.log 2>&1
rc=$?
tail -c 3000 gpurun_out/r5/bench1.log
exit $rc
