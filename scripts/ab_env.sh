#!/bin/bash
# Run one python script under several environment settings (one process each, own time limit),
# stopping at the first failure; one log per variant under OUT, the last stdout line echoed.
#   scripts/ab_env.sh OUT "python scripts/x.py args" "NAME:ENV=V ENV2=V" ...
O=$1; CMD=$2; shift 2
mkdir -p "$O"
for spec in "$@"; do
  name="${spec%%:*}"; envs="${spec#*:}"
  env $envs timeout -k 10 180 $CMD > "$O/$name.log" 2>&1
  rc=$?
  echo "[$name] $(grep -v amdgpu.ids "$O/$name.log" | tail -1)"
  if [ $rc -ne 0 ]; then echo "[$name] rc=$rc"; exit $rc; fi
done
