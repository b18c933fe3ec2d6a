#!/bin/bash
# Retry a gpurun call only when the infrastructure reports a transient failure
# (box lost while being prepared / no box free: nothing ran, nothing charged).
# Usage: tools/gpurun_retry.sh <outfile> <timeout> '<command>'
out=$1; lim=$2; cmd=$3
for i in 1 2 3 4 5 6; do
  timeout $((lim + 900)) /usr/local/graft/bin/gpurun --timeout "$lim" -- "$cmd" > "$out" 2>&1
  rc=$?
  if grep -q "status=transient\|backing off" "$out" || [ $rc -eq 3 ]; then
    echo "attempt $i transient, waiting" >> "$out.attempts"; sleep $((30 * i)); continue
  fi
  break
done
cat "$out"
