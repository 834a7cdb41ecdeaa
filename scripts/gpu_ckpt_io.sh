#!/bin/bash
# Native checkpoint I/O at the bench size (512^3 fp64 = 1.07 GB shard): write after 8
# steps, restart on 1 and 2 ranks (socket) for 8 more; wall time of each run (process
# start, field setup, 8 steps and the file I/O included).
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
D=$(mktemp -d /tmp/advdiff_ck.XXXXXX)
timeout -k 10 300 python -u - "$D" <<'PY'
import os, subprocess, sys, time
sys.path.insert(0, ".")
from multigpu_advectiondiffusion_amd.launch import launch
d = sys.argv[1]
A = "1 1 1 1 512 512 512 8 --ic sine".split()
env = dict(os.environ, RANK="0", WORLD_SIZE="1")
def run(tag, extra):
    t = time.time()
    subprocess.run(["bin/diffusion3d"] + A + extra, env=env, check=True, stdout=subprocess.DEVNULL)
    print(f"{tag}: {time.time() - t:.2f} s wall", flush=True)
run("plain run, 1 rank", [])
run("run + checkpoint write, 1 rank", ["--checkpoint", f"{d}/h"])
print("shard bytes:", sum(os.path.getsize(os.path.join(d, f)) for f in os.listdir(d)), flush=True)
run("restart + run, 1 rank", ["--restart", f"{d}/h"])
t = time.time()
rc = launch(2, ["diffusion3d"] + A + ["--restart", f"{d}/h", "--transport", "socket"], native=True, timeout=150)
print(f"restart + run, 2 ranks (socket): rc {rc}, {time.time() - t:.2f} s wall", flush=True)
PY
rc=$?
rm -rf "$D"
exit $rc
