#!/bin/bash
# Round-3 measurements: 2-D WENO5 kernel versions (v2 barrier-free vs v1 row tile) on the
# reference's 400x406 and large grids, and the multi-rank host-issue vs GPU-time rows.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
for v in 2 1; do
  ADVDIFF_B2_VER=$v timeout -k 10 300 python -u bench/small2d.py burgers2d > gpurun_out/small2d_v$v.log 2>&1 || { echo "small2d v$v FAILED"; tail -20 gpurun_out/small2d_v$v.log; exit 1; }
  echo "v$v: $(tail -1 gpurun_out/small2d_v$v.log)"
done
timeout -k 10 600 python -u bench/multigpu_graph.py > gpurun_out/multigpu_graph.log 2>&1 || { echo "multigpu_graph FAILED"; tail -30 gpurun_out/multigpu_graph.log; exit 1; }
grep '^{' gpurun_out/multigpu_graph.log
