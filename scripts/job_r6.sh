#!/bin/bash
# Round-6 GPU jobs: bash scripts/job_r6.sh NAME (one gpurun call each; steps via gpu_steps.sh)
R="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
SH="ADVDIFF_SHARE_GPU=1 GPU_MAX_HW_QUEUES=2 ADVDIFF_IPC_TIMEOUT_S=60"
PT="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
case "$1" in
  rehearsal)
    bash scripts/gpu_steps.sh r6/rehearsal \
      "reh2_hang|400|$SH ADVDIFF_FAULT=hang:heat:2x1x1/ipc $R --nproc-per-node 2 --master-port 29602 bench.py --gpus 2 --steps 10 --warmup 3 --sustained-steps 0 --preflight-cand-s 30" \
      "reh4|450|$SH $R --nproc-per-node 4 --master-port 29604 bench.py --gpus 4 --steps 10 --warmup 3 --sustained-steps 0" \
      "kernels|600|$PT tests/test_kernels_gpu.py tests/test_weno7_lsrk_gpu.py tests/test_fused_step_gpu.py" ;;
  suite)  # the driver's round-end tiers: GPU tests, smoke, bench
    bash scripts/gpu_steps.sh r6/suite \
      "pytest_gpu|900|$PT -m gpu tests" \
      "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
      "bench|600|python -u bench.py" ;;
  *) echo "unknown job $1"; exit 2 ;;
esac
