#!/bin/bash
# Round 4: native runtime changes (2 fields, watchdog, dry staging) + the WENO5 v9 tile-row
# variant: its numerics tests, then the A/B against the 64-wide tiles.
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
step kernels_b3 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "burgers3d"
step native_tests 600 python -u -m pytest tests/test_native_apps_gpu.py -x -q --timeout 180 --timeout-method thread
step burgers_tile_ab 600 python bench/burgers_tile_ab.py --rounds 2
