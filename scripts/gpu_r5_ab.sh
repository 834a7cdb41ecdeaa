#!/bin/bash
# Round-5 A/Bs of the round-4 kernel defaults (each step bounded; any failure ends the
# script): FD2 two-step vs one-step launch, packed vs unpacked fp32 WENO5 vs fp64, fp32
# heat tiles, 3-D rate vs size (Burgers 256^3 vs 512^3).
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/r5/ab
mkdir -p "$out"
export PYTHONUNBUFFERED=1
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name"
  timeout -k 10 "$lim" "$@" > "$out/$name.log" 2>&1
  local rc=$?
  grep -v amdgpu.ids "$out/$name.log" | tail -n 12
  if [ $rc -ne 0 ]; then echo "$name rc=$rc: stopping"; exit $rc; fi
}
for s in ${AB_STEPS:-step2 fp32weno fp32heat sizes}; do
  case $s in
    step2) step step2_ab 300 python bench/step2_ab.py --sizes 512,1024 --rounds 4 ;;
    fp32weno) step burgers_fp32_ab 300 python bench/burgers_fp32_ab.py --sizes 256,512 --rounds 3 ;;
    fp32heat) step step_fp32_ab 240 python bench/step_fp32_ab.py --n 512 --rounds 3 ;;
    sizes) step sizes3d 400 python bench/sizes3d.py --max 1024 --burgers-max 512 ;;
    tile) step burgers_tile_ab 500 python bench/burgers_tile_ab.py --rounds 2 ;;
  esac
done
echo done
