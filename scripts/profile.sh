#!/bin/bash
# rocprofv3 kernel-trace + stats of a short bench run (no PMC counters here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/${PROF_NAME:-bench} -o run -- \
  python3 bench.py ${BENCH_ARGS:---steps 20 --warmup 3} > gpurun_out/prof_${PROF_NAME:-bench}.log 2>&1
rc=$?; tail -3 gpurun_out/prof_${PROF_NAME:-bench}.log; echo "rocprof exit $rc"
find gpurun_out/prof -name "*stats*" | head
exit $rc
