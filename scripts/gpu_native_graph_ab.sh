#!/bin/bash
# Native engine: hipGraph vs eager stepping, alternated (each run its own process).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
: > gpurun_out/native_graph_ab.log
for r in 1 2 3; do
  for g in --graph --no-graph; do
    for o in 4 2; do
      t=$(RANK=0 WORLD_SIZE=1 timeout -k 10 120 bin/diffusion3d 1 1 1 1 512 512 512 ${ITERS:-200} --ic sine --order $o $g 2>&1 | grep "MLUPS (cells" | awk '{print $NF}') || exit 1
      echo "round $r order $o $g MLUPS $t" | tee -a gpurun_out/native_graph_ab.log
    done
  done
done
