#!/bin/bash
# Build variant libadvdiff.so files (bench/ab_libs/<name>.so) whose kernel objects are
# compiled with extra compiler flags, for in-process A/Bs (bench/ab_step.py,
# bench/ab_burgers.py).  Usage: scripts/build_ab_libs.sh name "flags" [name "flags" ...]
set -e
cd "$(dirname "$0")/../csrc"
ROCM=${ROCM:-/opt/rocm}
out=../bench/ab_libs
mkdir -p $out build/ab
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  objs=()
  for k in diffusion diffusion_fused diffusion2d_fused burgers aux ipc; do
    $ROCM/bin/hipcc -O3 --offload-arch=gfx950 -std=c++20 -fPIC -Iinclude -Ikernels -Wall \
      -Wno-unused-function $flags -c kernels/$k.hip -o build/ab/${name}_$k.o &
    objs+=(build/ab/${name}_$k.o)
  done
  wait
  $ROCM/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/$name.so "${objs[@]}" build/srchash.o
  echo "built $out/$name.so ($flags)"
done
