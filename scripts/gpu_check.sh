#!/bin/bash
# GPU validation run used with gpurun: tests, smoke, short bench.
# Stops at the first fault-like exit (abort/segv/timeout); plain test failures (exit 1)
# do not stop the later steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
ok_or_stop() { # $1 = exit code
  case "$1" in 0|1) return 0;; *) echo "fault-like exit $1: stopping"; exit "$1";; esac
}
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log; tail -15 gpurun_out/pytest_gpu.log; ok_or_stop $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; cat gpurun_out/smoke.log | tail -5; ok_or_stop $rc
timeout -k 10 600 python bench.py ${BENCH_ARGS:---steps 20 --warmup 3} > gpurun_out/bench.log 2>&1
rc=$?; tail -5 gpurun_out/bench.log; ok_or_stop $rc
