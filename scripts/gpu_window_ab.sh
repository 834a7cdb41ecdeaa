#!/bin/bash
# Headline-window A/B of fused-step variants: bench.py (20 steps after 5 warm-up, the
# driver's window) alternated between variants, each its own process.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
: > gpurun_out/window_ab.log
for r in 1 2 3 4; do
  for v in ${VARS:-3 23}; do
    ADVDIFF_STEP_VAR=$v timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-burgers \
      --sustained-steps 0 ${EXTRA:-} > gpurun_out/window_tmp.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/window_tmp.log; exit 1; }
    echo "var $v $(grep '^{' gpurun_out/window_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("fd2_7pt",{}).get("value"))')" | tee -a gpurun_out/window_ab.log
  done
done
