#!/bin/bash
# Dev helper: submit a gpurun command, re-submitting only while the pool reports no free slot or
# box (status=transient: nothing ran, nothing charged).  Usage: tools/gpurun_wait.sh <timeout> <script> <log>
T=$1; S=$2; LOG=$3
for i in $(seq 1 12); do
  timeout $((T + 900)) /usr/local/graft/bin/gpurun --timeout "$T" -- bash "$S" > "$LOG" 2>&1
  if grep -q 'status=transient' "$LOG"; then sleep 100; continue; fi
  break
done
tail -2 "$LOG"
