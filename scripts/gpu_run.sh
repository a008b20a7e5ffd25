#!/bin/bash
# Run GPU steps in order; each step under its own time limit. A crash / abort / timeout stops the
# script (nothing more touches the GPU); a plain test failure (exit 1) lets later steps run.
# usage: scripts/gpu_run.sh "<name>:<seconds>:<command>" ...
mkdir -p gpurun_out
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== [$name] ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"; tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
