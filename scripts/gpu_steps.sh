#!/bin/bash
# Parameterised GPU job runner for gpurun (replaces the per-call job files of round 5).
#
#   bash scripts/gpu_steps.sh OUTDIR 'NAME|SECONDS|COMMAND' ['NAME|SECONDS|COMMAND' ...]
#
# Each step runs under its own `timeout -k 10 SECONDS`, writes gpurun_out/OUTDIR/NAME.log
# and prints its exit code and last lines.  The job stops at the first step that fails
# (any non-zero exit; KEEP_GOING=1 lets plain failures, exit 1, continue — never a fault,
# an abort, a segfault or a time limit).  A summary line per step goes to
# gpurun_out/OUTDIR/steps.txt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
out="gpurun_out/$1"; shift
mkdir -p "$out"
rc_all=0
for step in "$@"; do
  name="${step%%|*}"; rest="${step#*|}"
  secs="${rest%%|*}"; cmd="${rest#*|}"
  t0=$SECONDS
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  printf '%-24s rc=%-3s %5d s  %s\n' "$name" "$rc" "$((SECONDS - t0))" "$cmd" | tee -a "$out/steps.txt"
  tail -n "${TAIL:-6}" "$out/$name.log"
  if [ "$rc" -ne 0 ]; then
    rc_all=$rc
    if [ "${KEEP_GOING:-0}" = 1 ] && [ "$rc" -eq 1 ]; then continue; fi
    echo "stopping after step $name (exit $rc)"
    exit "$rc"
  fi
done
exit $rc_all
