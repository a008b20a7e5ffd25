#!/bin/bash
# Interleaved bench A/B of two source trees (the current one and ab/NAME, a copy of another
# commit with its own built library): scripts/ab_trees.sh NAME PAIRS
name=$1; pairs=${2:-3}
mkdir -p gpurun_out
summ() {
  python - "$1" "$2" << 'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(f"[{sys.argv[1]:10s}] {d['ms_per_step']:7.2f} ms/step  {d['value']/1e6:6.3f} Mframes/s", flush=True)
PY
}
for i in $(seq 1 $pairs); do
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 12 --warmup 3 > gpurun_out/abt_cur$i.log 2>&1 || { echo "cur rc=$?"; tail -5 gpurun_out/abt_cur$i.log; exit 1; }
  summ cur$i gpurun_out/abt_cur$i.log
  (cd ab/$name && timeout -k 10 240 python bench.py --no-cpu-baseline --steps 12 --warmup 3 > ../../gpurun_out/abt_${name}$i.log 2>&1) || { echo "$name rc=$?"; tail -5 gpurun_out/abt_${name}$i.log; exit 1; }
  summ $name$i gpurun_out/abt_${name}$i.log
done
