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
  shapes)  # multi-rank FD2 two-step (tests + slab-rank A/B), FD4 per-rank shapes (A/B + PMC)
    bash scripts/gpu_steps.sh r6/shapes \
      "mr2_tests|600|$PT tests/test_ipc_gpu.py -k 'two_step'" \
      "mr2_ab|300|python -u bench/mr_step2_ab.py" \
      "fd4_rank|300|python -u bench/mr_step2_ab.py --order 4" \
      "banded_fd4|400|python -u bench/banded_ab.py --cases 512,slab8,r4x2,1024 --orders 4" \
      "pmc_shapes|600|PMC_OUT=gpurun_out/r6/pmc_shapes PMC_TARGETS='fused slab8_int slab8_bnd r4x2_int cube1024' PMC_ARGS='--pitch 4,1' bash scripts/pmc_r5.sh" ;;
  reh8)  # the whole N = 8 flow (preflight, tuning, checks, deadline) with 8 ipc ranks on one GPU
    bash scripts/gpu_steps.sh r6/reh8 \
      "reh8|600|$SH $R --nproc-per-node 8 --master-port 29608 bench.py --gpus 8 --steps 10 --warmup 3" ;;
  rcclfail)  # RCCL refuses two ranks on one GPU: the real RCCL error path of the preflight
    bash scripts/gpu_steps.sh r6/rcclfail \
      "reh2_rccl|400|$SH $R --nproc-per-node 2 --master-port 29612 bench.py --gpus 2 --steps 10 --warmup 3 --sustained-steps 0 --transport rccl --no-burgers" ;;
  final)  # round-end tiers + evidence: GPU tests, smoke, bench, kernel-trace stats of the bench,
          # the slab-rank step schedules
    bash scripts/gpu_steps.sh r6/final \
      "pytest_gpu|900|$PT -m gpu tests" \
      "smoke|300|python -c 'import __graft_entry__ as g; g.smoke()'" \
      "bench|600|python -u bench.py" \
      "bench_prof|600|rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6/final/prof -o p -- python3 bench.py --steps 20 --no-burgers --sustained-steps 0" \
      "rank_steps|300|python -u bench/mr_step2_ab.py --order 4 && python -u bench/mr_step2_ab.py" ;;
  pmcb)  # counter row of the shipped WENO5-Z viscous stage (256^3 and 512^3)
    bash scripts/gpu_steps.sh r6/pmc_burgers \
      "pmc|600|PMC_OUT=gpurun_out/r6/pmc_burgers PMC_TARGETS='burgers burgers512' bash scripts/pmc_r5.sh" ;;
  fput)  # fused halo puts: bitwise tests (2-4 ipc ranks on the GPU), kernel-side A/B at the
         # slab-rank shapes, the N = 4 bench flow with the new candidate
    bash scripts/gpu_steps.sh r6/fput \
      "tests|600|$PT tests/test_ipc_gpu.py -k 'fused_put or slab_bitwise'" \
      "ab|300|python -u bench/fused_put_ab.py" \
      "reh4|450|$SH $R --nproc-per-node 4 --master-port 29604 bench.py --gpus 4 --steps 10 --warmup 3 --sustained-steps 0 --no-burgers" ;;
  bsplit)  # the Burgers stage's split cost at the slab-rank blocks; fused-put A/B re-check
    bash scripts/gpu_steps.sh r6/bsplit \
      "bsplit|300|python -u bench/burgers_split_ab.py" \
      "fput_ab|300|python -u bench/fused_put_ab.py" ;;
  fput2)  # fused halo puts in the WENO5 stage too: tests, kernel-side A/Bs, the N = 4 flow
    bash scripts/gpu_steps.sh r6/fput2 \
      "tests|600|$PT tests/test_ipc_gpu.py -k 'fused_put'" \
      "bsplit|300|python -u bench/burgers_split_ab.py" \
      "fput_ab|300|python -u bench/fused_put_ab.py" \
      "reh4|500|$SH $R --nproc-per-node 4 --master-port 29604 bench.py --gpus 4 --steps 10 --warmup 3 --sustained-steps 0" ;;
  fput3)  # native-engine fused halo puts + the N = 8 flow with the new candidates
    bash scripts/gpu_steps.sh r6/fput3 \
      "native|600|$PT tests/test_ipc_gpu.py -k 'native_fused_put or native_plain_overlap'" \
      "reh8|600|$SH $R --nproc-per-node 8 --master-port 29608 bench.py --gpus 8 --steps 10 --warmup 3" ;;
  fput4)  # fused puts with the top-band banded schedule: tests, A/B
    bash scripts/gpu_steps.sh r6/fput4 \
      "tests|600|ADVDIFF_STEP_BANDED=1 $PT tests/test_ipc_gpu.py -k 'fused_put'" \
      "ab|300|python -u bench/fused_put_ab.py" ;;
  fput5)  # fused puts over the striped exchange: tests (4-5 ranks, shared links), N = 8 flow
    bash scripts/gpu_steps.sh r6/fput5 \
      "tests|600|$PT tests/test_ipc_gpu.py -k 'fused_put'" \
      "reh8|600|$SH $R --nproc-per-node 8 --master-port 29608 bench.py --gpus 8 --steps 10 --warmup 3" ;;
  gap)  # the bench's Burgers window vs the rate tool: build path or thermal state
    bash scripts/gpu_steps.sh r6/burgers_gap "gap|300|python -u bench/burgers_bench_gap.py" ;;
  own)  # WENO5 v9 staging the own cell from the register column: kernel A/B (two builds in
        # one process, bitwise compared) and in-solver rates (alternating processes)
    A=bench/ab_libs/libadvdiff_base.so; B=bench/ab_libs/${OWN_LIB:-libadvdiff_own2.so}
    RATE="ADVDIFF_ALLOW_STALE=1 python -u bench/burgers3d_rate.py"
    bash scripts/gpu_steps.sh r6/${OWN_OUT:-own2} \
      "tests|600|$PT tests/test_kernels_gpu.py tests/test_weno7_lsrk_gpu.py tests/test_pitch_gpu.py -k 'burgers or b3 or weno'" \
      "kernel256|300|python -u bench/ab_burgers.py $A $B --n 256 --rounds 7" \
      "kernel512|300|python -u bench/ab_burgers.py $A $B --n 512 --rounds 5 --reps 20" \
      "kernel256_fp32|300|python -u bench/ab_burgers.py $A $B --n 256 --rounds 7 --fp32" \
      "solver256|600|for r in 1 2 3; do ADVDIFF_LIB=$A $RATE 256 && ADVDIFF_LIB=$B $RATE 256 || exit 1; done" \
      "solver512|600|for r in 1 2; do ADVDIFF_LIB=$A $RATE 512 && ADVDIFF_LIB=$B $RATE 512 || exit 1; done" ;;
  *) echo "unknown job $1"; exit 2 ;;
esac
