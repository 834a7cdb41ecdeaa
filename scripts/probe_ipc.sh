#!/bin/bash
# Device-path probes on the GPU box (bench/native/ipc_probe.hip): memset ordering, and
# two processes on one GPU exchanging through hipIpc-mapped buffers + device flags.
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/probe
mkdir -p $out
timeout -k 10 120 bench/native/ipc_probe memset 20 > $out/memset.log 2>&1 || { echo "memset probe rc=$?"; exit 1; }
cat $out/memset.log
for put in 0 1; do
  d=$(mktemp -d)
  timeout -k 10 90 bench/native/ipc_probe ipc 0 $d 300 $put > $out/ipc_r0_put$put.log 2>&1 &
  p0=$!
  timeout -k 10 90 bench/native/ipc_probe ipc 1 $d 300 $put > $out/ipc_r1_put$put.log 2>&1 &
  p1=$!
  wait $p0; r0=$?
  wait $p1; r1=$?
  cat $out/ipc_r0_put$put.log $out/ipc_r1_put$put.log
  echo "put=$put rc: $r0 $r1"
  if [ $r0 -ne 0 ] || [ $r1 -ne 0 ]; then exit 1; fi
done
