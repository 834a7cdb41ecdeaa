#!/bin/bash
# Round 5: the self-launched N > 1 bench on the box's ONE GPU (ranks share it; the times
# are not scaling numbers): transport tuner with the comm-stream boundary as the ipc
# default, ipc preflight, bitwise N-rank-vs-1-GPU checks and the Burgers torch-reference
# check on every rank.  Each step bounded; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out/r5
export ADVDIFF_SHARE_GPU=1 GPU_MAX_HW_QUEUES=2 ADVDIFF_IPC_TIMEOUT_S=60 ADVDIFF_TRANSPORT=ipc
for n in ${NS:-2 4}; do
  echo "== N=$n"
  timeout -k 10 ${LIMIT:-500} python bench.py --gpus $n --steps 10 --warmup 3 --sustained-steps 0 \
    ${BENCH_ARGS:-} > gpurun_out/r5/rehearsal_n$n.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "N=$n FAILED rc=$rc"; tail -40 gpurun_out/r5/rehearsal_n$n.log; exit $rc; fi
  grep '^{' gpurun_out/r5/rehearsal_n$n.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('n_gpus','value','halo_transport','transport_trials_ms_per_step','bitwise_vs_1gpu','ipc_preflight','rccl_world','config')}); print('fd2', r['fd2_7pt']); print('burgers', {k: r['burgers3d'].get(k) for k in ('value','halo_transport','transport_trials_ms_per_step','linf_vs_torch','reference_check')})"
done
