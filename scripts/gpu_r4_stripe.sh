#!/bin/bash
# Round 4: striped ipc exchange (GPU bitwise tests with ranks sharing the GPU), then the
# self-launched 8-rank bench rehearsal whose tuner sees the ipc+stripe candidate.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
step() { # name seconds cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ]; then echo "$name FAILED rc=$rc"; exit $rc; fi
}
step step2_tests 300 python -u -m pytest tests/test_fused_step_gpu.py -x -v --timeout 120 --timeout-method thread -k "two_step"
step native_step2 300 python -u -m pytest tests/test_native_apps_gpu.py -x -v --timeout 120 --timeout-method thread -k "two_step"
step burgers_det 300 python bench/burgers_determinism.py --reps 3
step step2_ab 300 python bench/step2_ab.py --rounds 4
step packed_tests 400 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "packed or burgers3d_stage or tile_rows"
step fp32_pack_ab 300 python bench/burgers_fp32_ab.py --rounds 4
step ipc_tests2 500 python -u -m pytest tests/test_ipc_gpu.py -x -v --timeout 150 --timeout-method thread -k "striped or preflight or boundary_stream"
step native_ipc 400 python -u -m pytest tests/test_native_apps_gpu.py tests/test_ipc_gpu.py -x -v --timeout 150 --timeout-method thread -k "native and ipc"
step fp32_tiles 300 python bench/step_fp32_ab.py --rounds 4
step burgers_chunks_ab 600 python bench/burgers_tile_ab.py --rounds 2 --variants "B3_CHUNKS=0 B3_CHUNKS=1"
step split_conc 200 python bench/split_overhead.py --reps 20
step bench1 500 python bench.py --steps 20 --warmup 5
export ADVDIFF_SHARE_GPU=1 GPU_MAX_HW_QUEUES=2 ADVDIFF_IPC_TIMEOUT_S=60 ADVDIFF_TRANSPORT=ipc
step rehearsal_self_n8 900 python bench.py --gpus 8 --steps 10 --warmup 3 --sustained-steps 0 --no-fd2
grep '^{' gpurun_out/rehearsal_self_n8.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print({k: r.get(k) for k in ('n_gpus','value','halo_transport','transport_trials_ms_per_step','bitwise_vs_1gpu','ipc_preflight','halo_link_MB','config')}); print('burgers', {k: r['burgers3d'].get(k) for k in ('halo_transport','transport_trials_ms_per_step','pgrid')})"
