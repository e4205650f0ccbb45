#!/bin/bash
# usage (host side, not on the GPU box): tools/gpu_retry.sh OUTFILE TIMEOUT 'command'   — retries only when no box/slot was available (nothing ran)
OUT=$1; TO=$2; CMD=$3
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$OUT" 2>&1
  rc=$?
  if grep -q "status=transient" "$OUT" && grep -q "nothing was charged\|retry in a few minutes\|retry$\|stopped responding while being prepared" "$OUT"; then
    echo "[retry $i: transient, rc=$rc]" >> "$OUT.retries"; sleep 120; continue
  fi
  break
done
echo "[done rc=$rc]" >> "$OUT"
