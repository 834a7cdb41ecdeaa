#!/bin/bash
# bench.py (the driver's contract, defaults) repeated back to back: the run-to-run spread of
# the 20-step window on one box.
cd "$(dirname "$0")/.." || exit 1
mkdir -p gpurun_out
: > gpurun_out/bench_repeat.log
for r in 1 2 3 4 5; do
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_tmp.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/bench_tmp.log; exit 1; }
  grep '^{' gpurun_out/bench_tmp.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({"run": '$r', "fd4_window": d["value"], "fd4_sustained": d["sustained"]["value"], "fd2_window": d["fd2_7pt"]["value"], "burgers_window": d["burgers3d"]["value"], "burgers_sustained": d["burgers3d"]["sustained"]["value"]}))' | tee -a gpurun_out/bench_repeat.log
done
