#!/bin/bash
# The N > 1 bench flow (decomposition tuning, halo diagnostics, Burgers, JSON line) with
# N ipc ranks sharing the box's ONE GPU (device puts + flags, graph-replayed steps).  Times
# are NOT scaling numbers (the ranks' kernels share one GPU); this checks the flow.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
export ADVDIFF_SHARE_GPU=1 ADVDIFF_TRANSPORT=ipc GPU_MAX_HW_QUEUES=2 ADVDIFF_IPC_TIMEOUT_S=60
for n in ${NS:-2 4 8}; do
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port $((29600 + n)) bench.py --gpus $n --steps 10 \
    --warmup 3 --sustained-steps 0 > gpurun_out/rehearsal_ipc_n$n.log 2>&1 || { echo "N=$n FAILED"; tail -40 gpurun_out/rehearsal_ipc_n$n.log; exit 1; }
  echo "N=$n ok"; grep '^{' gpurun_out/rehearsal_ipc_n$n.log | tail -1
done
