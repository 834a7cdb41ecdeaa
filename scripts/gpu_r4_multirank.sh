#!/bin/bash
# Round 4: the N > 1 bench machinery on the box's ONE GPU (ranks share it; times are not
# scaling numbers): ipc kernels' tests, the single-GPU bench, the self-launched bench with
# the transport tuner + ipc preflight + bitwise N-rank-vs-1-GPU checks, and per-rank
# rocprofv3 traces through launch.py --profile.  Every GPU step has its own time limit and
# the steps are chained: a fault or timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
set -o pipefail
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; exit $rc; fi
}
step ipc_tests 400 python -u -m pytest tests/test_ipc_gpu.py -x -q --timeout 120 --timeout-method thread
step bench1 300 python bench.py --steps 20 --warmup 5
export ADVDIFF_SHARE_GPU=1 GPU_MAX_HW_QUEUES=2 ADVDIFF_IPC_TIMEOUT_S=60 ADVDIFF_TRANSPORT=ipc
for n in ${NS:-2 4}; do
  step rehearsal_self_n$n 500 python bench.py --gpus $n --steps 10 --warmup 3 --sustained-steps 0
  grep '^{' gpurun_out/rehearsal_self_n$n.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('n_gpus','value','halo_transport','transport_trials_ms_per_step','bitwise_vs_1gpu','ipc_preflight','rccl_world')}); print('burgers', {k: r['burgers3d'].get(k) for k in ('halo_transport','transport_trials_ms_per_step')})"
done
step prof_ranks 300 python -m multigpu_advectiondiffusion_amd.launch -np 2 --profile gpurun_out/prof_ranks diffusion3d 1 1 1 1 512 512 512 40 --ic sine --transport ipc
python bench/trace_overlap.py gpurun_out/prof_ranks --md gpurun_out/prof_ranks_overlap.md
