#!/bin/bash
# Development helper (runs here, not on the box): submit one gpurun call, resubmitting it only when gpurun reports a
# transient infrastructure status (no slot / box lost while being prepared: nothing ran, nothing charged), at most
# 6 times, 2 minutes apart. Usage: tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
OUT=$1; TO=$2; CMD=$3
for i in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if grep -q 'status=transient' "$OUT" && grep -q 'run 0.0s' "$OUT"; then
    echo "[retry $i: transient]" >> "$OUT.tries"; sleep 120; continue
  fi
  exit $rc
done
exit 3
