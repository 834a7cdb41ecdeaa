#!/bin/bash
# Kernel trace of a 2-rank native ipc heat run (the N = 8 per-rank block 1024x1024x128,
# ranks sharing the box's GPU): do the halo puts run beside the rank's own interior launch?
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp ADVDIFF_SHARE_GPU=1 GPU_MAX_HW_QUEUES=2 ADVDIFF_IPC_TIMEOUT_S=60
tag=${TAG:-graph}
mkdir -p gpurun_out/ipc_trace_$tag
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ipc_trace_$tag -o run -- \
  python3 -m multigpu_advectiondiffusion_amd.launch -np 2 --native diffusion3d 1 1 1 1 1024 1024 256 24 \
  --ic sine --transport ipc ${EXTRA:-} > gpurun_out/ipc_trace_$tag.log 2>&1 || { echo "trace run failed"; tail -20 gpurun_out/ipc_trace_$tag.log; exit 1; }
python3 bench/trace_overlap.py gpurun_out/ipc_trace_$tag --md gpurun_out/ipc_overlap_$tag.md
