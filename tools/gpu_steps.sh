#!/bin/bash
# Run GPU steps in order; each under its own timeout. Stop at the first fault-like exit
# (abort 134, segfault 139, timeout 124/137, signal-killed >128) — never retry a GPU step.
# Usage: tools/gpu_steps.sh "<secs>|<name>|<cmd>" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
for spec in "$@"; do
  secs="${spec%%|*}"; rest="${spec#*|}"; name="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] $(date +%T) timeout=${secs}s: $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/${name}.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc $(date +%T)"
  tail -n 25 "gpurun_out/${name}.log"
  if [ $rc -ge 124 ]; then
    echo "=== stopping: fault-like exit $rc in $name"
    exit $rc
  fi
  [ $rc -ne 0 ] && status=$rc
done
exit $status
