#!/bin/bash
# Per-rank overlap of the halo puts with the rank's own stencil launches (rocprofv3 kernel
# trace per rank via launch.py --profile), 2 ipc ranks sharing the box's GPU, at the 8-GPU
# per-rank block shapes (heat 1024x1024x128, Burgers 512x512x64), the default overlapped
# path vs the boundary launch on the comm stream (ADVDIFF_BCOMM=1).
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/r5/overlap
rm -rf "$out"; mkdir -p "$out"
export ADVDIFF_SHARE_GPU=1 GPU_MAX_HW_QUEUES=2 ADVDIFF_IPC_TIMEOUT_S=20 PYTHONUNBUFFERED=1
L="python -m multigpu_advectiondiffusion_amd.launch -np 2 --timeout 240"
run() {  # name bcomm args...
  local name=$1 bc=$2; shift 2
  echo "== $name"
  ADVDIFF_BCOMM=$bc timeout -k 10 280 $L --profile "$out/$name" "$@" --transport ipc \
    > "$out/$name.log" 2>&1 || { echo "$name failed rc=$?"; tail -n 30 "$out/$name.log"; exit 1; }
  python bench/trace_overlap.py "$out/$name" --md "$out/$name.md"
  ADVDIFF_BCOMM=$bc timeout -k 10 200 $L "$@" --transport ipc > "$out/${name}_noprof.log" 2>&1 \
    || { echo "$name (no profiler) failed"; exit 1; }
  grep -i "time\|MLUPS" "$out/${name}_noprof.log" | head -8
}
run heat_plain 0 diffusion3d 1 1 1 1 1024 1024 256 40 --ic sine
run heat_bcomm 1 diffusion3d 1 1 1 1 1024 1024 256 40 --ic sine
run burg_plain 0 burgers3d 0.047 0.3 2 2 2 512 512 128
run burg_bcomm 1 burgers3d 0.047 0.3 2 2 2 512 512 128
echo done
