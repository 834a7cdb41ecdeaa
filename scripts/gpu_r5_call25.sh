#!/bin/bash
# round 5: the bench with the z schedule forced uniform vs measured (same box, alternating)
set -o pipefail
mkdir -p gpurun_out/r5
for i in 1 2; do
  for m in 0 auto; do
    if [ $m = auto ]; then unset ADVDIFF_STEP_BANDED; else export ADVDIFF_STEP_BANDED=$m; fi
    ADVDIFF_STEP_BANDS_LOG=1 timeout -k 10 200 python -u bench.py --no-burgers > gpurun_out/r5/bench_sched_${m}_$i.log 2>&1 || exit 1
    echo "$m $i $(grep advdiff gpurun_out/r5/bench_sched_${m}_$i.log | tr '\n' ' ')"
    grep -o '"value": [0-9.]*, "unit": "MLUPS", "n_gpus"\|"fd2_7pt": {"value": [0-9.]*\|"sustained": {"steps": 200, "value": [0-9.]*' gpurun_out/r5/bench_sched_${m}_$i.log | tr '\n' ' '; echo
  done
done
