#!/bin/bash
# Run GPU steps in order, each under its own time limit; an ordinary failure (exit 1, e.g. a
# failing test) moves on to the next step, anything that smells of a fault or hang (timeout 124 /
# 137, abort 134, segfault 139, ...) stops the whole call so nothing else touches the GPU.
#   scripts/gpu_steps.sh OUT_DIR "SECONDS|command" ["SECONDS|command" ...]
out=$1
shift
mkdir -p "$out"
n=0
final=0
for spec in "$@"; do
  n=$((n + 1))
  secs=${spec%%|*}
  cmd=${spec#*|}
  echo "== step $n (${secs}s): $cmd" | tee -a "$out/steps.log"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/step$n.log" 2>&1
  rc=$?
  echo "== step $n rc=$rc" | tee -a "$out/steps.log"
  if [ $rc -ne 0 ]; then final=$rc; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping: step $n exited $rc" | tee -a "$out/steps.log"
    exit $rc
  fi
done
exit $final
