#!/bin/bash
# Round-5 boundary-stream diagnosis: each variant in its own bounded process; a variant
# that reports BAD (rc 1) is recorded and the next one runs; a timeout, abort or crash ends
# the script (nothing more runs on the GPU after it).
cd "$(dirname "$0")/.." || exit 1
out=gpurun_out/r5
mkdir -p "$out"
export ADVDIFF_IPC_TIMEOUT_S=5 PYTHONUNBUFFERED=1
run() {  # name hwq limit args...
  local name=$1 hwq=$2 lim=$3
  shift 3
  echo "== $name (GPU_MAX_HW_QUEUES=$hwq)"
  GPU_MAX_HW_QUEUES=$hwq timeout -k 10 "$lim" python scripts/diag_bstream.py "$@" \
    > "$out/diag_$name.log" 2>&1
  local rc=$?
  echo "   rc=$rc: $(tail -n 1 "$out/diag_$name.log")"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after rc=$rc"
    exit $rc
  fi
}
for v in ${DIAG_VARIANTS:-plain_graph comm_graph}; do
  m=${v%%_*}; g=${v#*_}
  run "$v" "${DIAG_HWQ:-2}" 150 "$m" "$g" 17
done
echo done
