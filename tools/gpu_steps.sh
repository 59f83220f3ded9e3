#!/bin/bash
# Run GPU steps one after another on the box, each under its own time limit; a step that ends in
# an assertion failure (rc 1, pytest 1) lets the next one run, but a fault, abort, segfault or time
# limit (rc 124 / 134 / 137 / 139, or anything >= 124) stops the call there.
#   bash tools/gpu_steps.sh "name:seconds:command" ...
# Output of step `name` goes to gpurun_out/<name>.log.
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
  echo "[step] $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[step] $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then
    echo "[step] $name ended by a fault / abort / time limit: stopping"
    exit $rc
  fi
done
