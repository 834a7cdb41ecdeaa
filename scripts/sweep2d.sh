#!/bin/bash
# 2-D fused-step chunking sweep on the reference's two 2-D heat grids (+ a large one).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "${SWEEP2D_CONFIGS[@]:-X=1}"; do
  echo "== $cfg"
  env ${cfg//+/ } timeout -k 10 120 python bench/reference_rows.py --only Diffusion-2D | cut -c1-120 || exit 1
done
