#!/bin/bash
# Run GPU steps in order on the gpurun box; each under its own time limit. Stop at the first step that
# crashes, aborts, faults or times out (exit codes other than 0/1); an ordinary test failure (1) does
# not stop the sequence. Logs go to gpurun_out/.
#   usage: tools/gpu_steps.sh "<name>:<seconds>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: step $name ended with rc=$rc"
    exit $rc
  fi
done
